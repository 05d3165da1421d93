#!/usr/bin/env bash
# Round 5 pass o: per-dispatch durations of the kd-tree build kernels (one C3-sized build), for the per-level split.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05o}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 $R/tools/kd_build_probe.py --reps 1 > "$OUT/probe.json" 2> "$OUT/probe.err"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
out = open(sys.argv[1] + "/kd_dispatches.txt", "w")
for r in rows:
    n = r["Kernel_Name"]
    if "kd_" in n:
        out.write(f"{n.split('(')[0][:40]:40s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:9.1f} us  grid {r.get('Grid_Size', r.get('Grid_Size_X', ''))}\n")
PY
rm -rf "$OUT/trace"

#!/usr/bin/env bash
# Round 5 pass q7 (study): q7 the orbit scan launched twice back to back (TILER_DEBUG_SCAN_TWICE in a study build,
# libANN_x.so): does the second launch run faster (instruction-cache / first-touch costs of the first)?  q7b: the
# study build without the 3 mirror members' sums (STUDY_M=0: the VALU share of the kernel).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05q7}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 $R/tools/percall_probe.py --scan-only --lib $R/tiler_amd/lib/ab/libANN_x.so > "$OUT/probe.json" 2> "$OUT/probe.err"
find "$OUT/trace" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/trace"
python3 - "$OUT/kernel_trace.csv" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "nn_scan_orbit" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
for name, a in (("1q", d[:31]), ("4q", d[31:62]), ("16q", d[62:])):
    print(name, "%.1f us" % (sum(a) / len(a)))
PY

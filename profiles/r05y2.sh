#!/usr/bin/env bash
# Round 5 pass y2 (study): where a lone per-tile call's time goes -- HIP API, copy and kernel timeline of the
# per-call probe's lone phase (C3 keyframe handle), from rocprofv3 runtime + kernel + copy traces (no counters).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05y2}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run --output-format csv -- python3 $R/tools/percall_probe.py --queries 512 > "$OUT/probe.json" 2> "$OUT/probe.err"
for f in hip_api_trace kernel_trace memory_copy_trace; do find "$OUT/trace" -name "*${f}.csv" -exec cp {} "$OUT/$f.csv" \; ; done
rm -rf "$OUT/trace"
python3 $R/tools/lone_timeline.py "$OUT" > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"

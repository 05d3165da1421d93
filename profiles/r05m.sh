#!/usr/bin/env bash
# Round 5 pass m: per-kernel split of the kd-tree build after r05l (kernel stats of tools/kd_build_probe.py).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05m}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $R/tools/kd_build_probe.py --reps 3 > "$OUT/probe.json" 2> "$OUT/probe.err"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/trace"

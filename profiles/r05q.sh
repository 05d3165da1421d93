#!/usr/bin/env bash
# Round 5 pass q: kernel split of the per-call path (tools/percall_probe.py under the kernel tracer): the small-batch
# scan vs its merge + pruning-check kernel vs the rest.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05q}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $R/tools/percall_probe.py --queries 2048 --scan-only > "$OUT/probe.json" 2> "$OUT/probe.err"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/trace"

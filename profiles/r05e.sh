#!/usr/bin/env bash
# Round 5 pass e: where the sustained encoder loop's GPU time goes -- a kernel trace of bench_encoder (10 keyframes,
# shot-local items, no overlap so every phase runs alone), summarised per kernel.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05e}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $R/bench_encoder.py --frames 240 --item-tiles 16384 --check-kf -1 --no-overlap > "$OUT/enc.json" 2> "$OUT/enc.err"
echo "trace done"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/trace"
head -30 "$OUT/kernel_stats.csv" | cut -c1-160

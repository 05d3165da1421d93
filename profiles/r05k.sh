#!/usr/bin/env bash
# Round 5 pass k: per-kernel cost of the encoder loop without overlap (each kernel alone on the chip): kernel stats
# of a 240-frame clip (10 keyframes), shot-local and whole-tileset items.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05k}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for items in 16384 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$items" -o run --output-format csv -- python3 $R/bench_encoder.py --frames 240 --item-tiles $items --check-kf -1 --no-overlap > "$OUT/enc_$items.json" 2> "$OUT/enc_$items.err"
  find "$OUT/trace_$items" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$items.csv" \;
  rm -rf "$OUT/trace_$items"
  echo "items $items done"
done

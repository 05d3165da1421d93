#!/usr/bin/env bash
# Round-3 pass zq: K-Modes move statistics per iteration at C4 (experiment build, TILER_KM_STATS): how many moves and
# groups the largest bin makes per iteration (input to the round-4 assignment plan).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zq
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
TILER_KM_STATS=1 timeout -k 10 300 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt.json" 2> "$OUT/gt.err" || true
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
grep km_stats "$OUT/gt.err" | tail -30

#!/usr/bin/env bash
# Round-3 pass q: K-Modes sequential-pass counters per iteration (experiment build, TILER_KM_STATS) at C4.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03q}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
TILER_KM_STATS=1 timeout -k 10 300 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_stats.json" 2> "$OUT/gt_stats.err" || true
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
grep km_stats "$OUT/gt_stats.err" | head -40

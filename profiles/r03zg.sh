#!/usr/bin/env bash
# Round-3 pass zg: where the K-Modes move passes spend their time -- experiment build, TILER_KM_STATS: per iteration
# the largest bin's shader-clock sums of staging, list builds, candidate fetch, group choice, apply and rescue; then
# the K-Modes GPU tests on the shipped build (the diagnostic adds only branches on a null pointer there).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zg
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
TILER_KM_STATS=1 timeout -k 10 300 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_stats.json" 2> "$OUT/gt_stats.err" || true
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
grep "km_clock" "$OUT/gt_stats.err" | head -30
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kmodes.py -m gpu -x -q --timeout 500 --timeout-method thread -k "not c4_full and not c5_shaped" > "$OUT/kmodes_tests.log" 2>&1
tail -1 "$OUT/kmodes_tests.log"

#!/usr/bin/env bash
# Round-3 pass z: K-Modes move pass with the candidates fetched by the selecting wave, cluster sizes in LDS (and the other-modalities tests) -- K-Modes /
# GlobalTiling / pipeline parity tests, the C4 line, then the per-iteration counters (experiment build).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03zb}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
python3 -c "import json; d=json.loads(open('$OUT/gt.json').read().strip().splitlines()[-1]); print('shipped', d['value'], d['phases'], d['cpu_baseline']['bins_mismatching_gpu'])"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
TILER_KM_STATS=1 timeout -k 10 300 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_stats.json" 2> "$OUT/gt_stats.err" || true
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
grep km_stats "$OUT/gt_stats.err" | head -6

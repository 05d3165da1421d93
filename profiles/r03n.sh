#!/usr/bin/env bash
# Round-3 pass n: K-Modes sequential pass with 32 concurrent moves of 16 lanes -- the K-Modes / GlobalTiling /
# pipeline parity tests, the C4 line, then 16 vs 80 lanes per move (experiment build, TILER_KM_SEQ_W).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03n}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "globaltiling done"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for w in 80 16; do
  TILER_KM_SEQ_W=$w timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_w$w.json" 2> "$OUT/gt_w$w.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_w$w.json').read().strip().splitlines()[-1]); print('w $w', d['value'], d['phases'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
echo "w ab done"

#!/usr/bin/env bash
# Round-3 pass k: K-Modes with the persistent farthest-first launch -- the K-Modes / GlobalTiling / pipeline parity
# tests, the C4 line, then per-launch vs persistent rounds (experiment build, TILER_KM_FF=0/1).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03k}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "globaltiling done"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for m in 0 1; do
  TILER_KM_FF=$m timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_ff$m.json" 2> "$OUT/gt_ff$m.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_ff$m.json').read().strip().splitlines()[-1]); print('ff $m', d['value'], d['phases'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
echo "ff ab done"

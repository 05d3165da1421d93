#!/usr/bin/env bash
# Round-3 pass o: K-Modes with the <= 16-modality assignment (kmb_assign16) and the 32-move sequential pass --
# the K-Modes / GlobalTiling / pipeline parity tests, the C4 line, then A/B in the experiment build:
# the general assignment (TILER_KM_A16=0) and 80 lanes per move (TILER_KM_SEQ_W=80).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03o}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "globaltiling done"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in "TILER_KM_A16=0" "TILER_KM_SEQ_W=80" "TILER_KM_A16=1"; do
  env $v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_$v.json" 2> "$OUT/gt_$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['phases'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
echo "ab done"

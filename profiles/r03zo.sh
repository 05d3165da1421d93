#!/usr/bin/env bash
# Round-3 pass zo: farthest-first with the selection after the barrier (experiment build, TILER_KM_FF=2) vs the shipped
# persistent kernel: C4 K-Modes (timers off; digest of labels + centroids), then the K-Modes GPU tests on the variant.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zo
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 1 2 1 2; do
  TILER_KM_FF=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_ff$v.json" 2> "$OUT/gt_ff$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_ff$v.json').read().strip().splitlines()[-1]); print('FF $v', d['value'], d['digest'], d['phases']['kmodes_init'])"
done
TILER_KM_FF=2 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kmodes.py -m gpu -x -v --timeout 400 --timeout-method thread > "$OUT/tests_ff2.log" 2>&1
tail -2 "$OUT/tests_ff2.log"
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

#!/usr/bin/env bash
# Round-3 pass zh: K-Modes move passes split into a decision pass (one workgroup per bin: the move sequence, labels,
# sizes) and an attribute pass (kmb_seq_apply, 10 workgroups per bin) -- the K-Modes / GlobalTiling / pipeline tests,
# the C4 line, then A/B in the experiment build (TILER_KM_APPLY=0: decided and applied by one workgroup).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zh
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
python3 -c "import json; d=json.loads(open('$OUT/gt.json').read().strip().splitlines()[-1]); print('shipped', d['value'], d['phases'], d['cpu_baseline']['bins_mismatching_gpu'])"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in "TILER_KM_APPLY=0" "TILER_KM_APPLY=1"; do
  env $v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_$v.json" 2> "$OUT/gt_$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['phases'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

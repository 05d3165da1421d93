#!/usr/bin/env bash
# Round-3 pass zt: K-Modes decision pass with a 64-candidate window (experiment build, TILER_KM_DW=8) vs 32 (shipped);
# C4 timed with the timers off, digest must not change (r03zu: after the attribute pass loops over groups of more than 32 moves).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03zt}
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 16 8 16 8; do
  TILER_KM_DW=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_w$v.json" 2> "$OUT/gt_w$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_w$v.json').read().strip().splitlines()[-1]); print('DW $v', d['value'], d['digest'], d['phases']['kmodes_seq'], d['phases']['kmodes_apply'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py -m gpu -x -v --timeout 400 --timeout-method thread > "$OUT/tests_shipped.log" 2>&1
tail -1 "$OUT/tests_shipped.log"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt_shipped.json" 2> "$OUT/gt_shipped.err"
python3 -c "import json; d=json.loads(open('$OUT/gt_shipped.json').read().strip().splitlines()[-1]); print('shipped', d['value'], d['digest'], d['cpu_baseline']['bins_mismatching_gpu'])"

#!/usr/bin/env bash
# Round-3 pass zi: K-Modes attribute pass over 5 / 10 / 20 / 40 workgroups per bin (experiment build, TILER_KM_SLICES),
# decision and attribute passes timed apart; then the shipped C4 line.  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zi
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
python3 -c "import json; d=json.loads(open('$OUT/gt.json').read().strip().splitlines()[-1]); print('shipped', d['value'], d['phases'], d['cpu_baseline']['bins_mismatching_gpu'])"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 5 10 20 40 10; do
  TILER_KM_SLICES=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_s$v.json" 2> "$OUT/gt_s$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_s$v.json').read().strip().splitlines()[-1]); print('slices $v', d['value'], d['phases'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

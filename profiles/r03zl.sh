#!/usr/bin/env bash
# Round-3 pass zl: kmb_assign16 over 1 / 2 / 4 / 8 / 16 workgroups per work item (experiment build, TILER_KM_ASUB), C4 K-Modes timed
# with the timers off; the digest of labels + centroids must not change.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zl
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 4 1 2 8 16 4 8 16; do
  TILER_KM_ASUB=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_a$v.json" 2> "$OUT/gt_a$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_a$v.json').read().strip().splitlines()[-1]); print('ASUB $v', d['value'], d['digest'], d['phases']['kmodes_assign'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

#!/usr/bin/env bash
# Round-3 pass zk: kmb_assign16 with 1 / 2 / 4 points per thread (experiment build, TILER_KM_A16P), C4 K-Modes timed
# with the timers off; the digest of labels + centroids must not change.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zk
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 1 2 4 1 2 4; do
  TILER_KM_A16P=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_p$v.json" 2> "$OUT/gt_p$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_p$v.json').read().strip().splitlines()[-1]); print('P $v', d['value'], d['digest'], d['phases']['kmodes_assign'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

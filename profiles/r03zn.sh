#!/usr/bin/env bash
# Round-3 pass zn: kmb_assign16 with the next centroid's LDS row prefetched (experiment build, TILER_KM_A16PF=1) vs
# the shipped loop, C4 K-Modes timed with the timers off; the digest of labels + centroids must not change.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zn
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 0 1 0 1 0 1; do
  TILER_KM_A16PF=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_pf$v.json" 2> "$OUT/gt_pf$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_pf$v.json').read().strip().splitlines()[-1]); print('PF $v', d['value'], d['digest'], d['phases']['kmodes_assign'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

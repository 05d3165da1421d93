#!/usr/bin/env bash
# Round-3 pass zw: K-Modes decision pass in one 1024-thread workgroup per bin (experiment build, TILER_KM_DNT=1024) vs 512 (shipped);
# C4 timed with the timers off, digest must not change (r03zu: after the attribute pass loops over groups of more than 32 moves).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03zw}
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 512 1024 512 1024; do
  TILER_KM_DNT=$v timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_n$v.json" 2> "$OUT/gt_n$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_n$v.json').read().strip().splitlines()[-1]); print('DNT $v', d['value'], d['digest'], d['phases']['kmodes_seq'], d['phases']['kmodes_apply'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

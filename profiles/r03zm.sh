#!/usr/bin/env bash
# Round-3 pass zm: kmb_assign16 with G groups of 256 threads per workgroup (experiment build, TILER_KM_A16G) and
# TILER_KM_ASUB slices per item, C4 K-Modes timed with the timers off; the digest of labels + centroids must not change.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zm
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in 4:1 4:2 4:4 8:2 8:4 16:4 4:1 4:2 4:4 8:4; do
  a=${v%:*}; g=${v#*:}
  TILER_KM_ASUB=$a TILER_KM_A16G=$g timeout -k 10 200 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_$a.$g.json" 2> "$OUT/gt_$a.$g.err"
  python3 -c "import json; d=json.loads(open('$OUT/gt_$a.$g.json').read().strip().splitlines()[-1]); print('ASUB $a G $g', d['value'], d['digest'], d['phases']['kmodes_assign'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

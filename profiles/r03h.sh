#!/usr/bin/env bash
# Round-3 pass h: C4 GlobalTiling with the per-launch K-Modes (default again), the sustained loop with shot-local
# items, then the generic 16x16x32 shortlist QB 4 vs 5 (experiment build) on a 4-keyframe clip.  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03h}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "globaltiling done"
timeout -k 10 300 python3 -u bench_encoder.py --check-kf -1 --item-tiles 16384 > "$OUT/enc_local.json" 2> "$OUT/enc_local.err"
echo "encoder local done"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for qb in 4 5 4 5; do
  TILER_SL16_QB=$qb timeout -k 10 200 python3 -u bench_encoder.py --check-kf -1 --frames 96 --no-overlap > "$OUT/enc_qb$qb.json" 2> "$OUT/enc_qb$qb.err"
  python3 -c "import json; d=json.loads(open('$OUT/enc_qb$qb.json').read().strip().splitlines()[-1]); print('qb $qb', d['wall_s'], d['diag']['ft_kernels'].get('nn_shortlist'), d['out_digest'])"
done
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
echo "qb ab done"

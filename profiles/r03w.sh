#!/usr/bin/env bash
# Round-3 pass w: generic 16x16x32 shortlist with the A fragments two k-step pairs ahead (TILER_SL16_PF=2) vs one
# (experiment build), on the C3 step with the orbit kernels off (TILER_ORBIT=0: every query through the generic
# shortlist against 262,144 candidates); prints step time, shortlist average and the output digest.  set -e.
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r03w
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for pf in 1 2 1 2; do
  TILER_ORBIT=0 TILER_SL16_PF=$pf timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 --no-keyframes --no-dither \
    --no-smooth --no-globaltiling --no-palettes > gpurun_out/r03w/pf$pf.json 2> gpurun_out/r03w/pf$pf.err
  python3 -c "import json; d=json.loads(open('gpurun_out/r03w/pf$pf.json').read().strip().splitlines()[-1]); k=d['kernels']; print('pf $pf', d['ms_per_step'], k['nn_shortlist']['ms_avg'], k['nn_rescore']['ms_avg'], d['search_stats'].get('fallback_queries'), d['out_digest'])"
done

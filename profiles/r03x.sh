#!/usr/bin/env bash
# Round-3 pass x: generic 16x16x32 shortlist with the epilogue of each block deferred past the next block's first
# k-step pair (TILER_SL16_DEF=1) vs in place (experiment build), on the C3 step with the orbit kernels off
# (TILER_ORBIT=0: every query through the generic shortlist against 262,144 candidates).  set -e.
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r03x
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for d in 0 1 0 1; do
  TILER_ORBIT=0 TILER_SL16_DEF=$d timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 --no-keyframes --no-dither \
    --no-smooth --no-globaltiling --no-palettes > gpurun_out/r03x/def$d.json 2> gpurun_out/r03x/def$d.err
  python3 -c "import json; d=json.loads(open('gpurun_out/r03x/def$d.json').read().strip().splitlines()[-1]); k=d['kernels']; print('def $d', d['ms_per_step'], k['nn_shortlist']['ms_avg'], k['nn_rescore']['ms_avg'], d['search_stats'].get('fallback_queries'), d['out_digest'])"
done

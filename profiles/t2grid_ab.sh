#!/usr/bin/env bash
# A/B of the orbit tier-2 grid (experiment build: TILER_T2_X query-group columns x TILER_T2_NSPLIT candidate splits)
# on the C3 bench step; prints step, collect average, tier-2 count and the output digest per variant.
set -eu
mkdir -p gpurun_out/t2
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in ${VARIANTS:-2:512 8:256 16:128 4:512 32:64 2:512}; do
  x=${v%%:*}; ns=${v##*:}
  TILER_T2_X=$x TILER_T2_NSPLIT=$ns timeout -k 10 200 python3 -u bench.py --no-cpu --steps 10 --no-keyframes --no-dither \
    --no-smooth --no-globaltiling --no-palettes > gpurun_out/t2/v$x-$ns.json 2> gpurun_out/t2/v$x-$ns.err
  python3 -c "import json; d=json.loads(open('gpurun_out/t2/v$x-$ns.json').read().strip().splitlines()[-1]); k=d['kernels']; print('x $x ns $ns', d['ms_per_step'], k['nn_orbit']['ms_avg'], k['nn_collect']['ms_avg'], k['nn_rescore2']['ms_avg'], d['search_stats'].get('fallback_queries'), d['out_digest'])"
done

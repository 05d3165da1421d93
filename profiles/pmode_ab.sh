#!/usr/bin/env bash
# A/B of shortlist kernel variants (experiment build, TILER_ORBIT_PMODE; modes 0 and >= 3 are valid): per mode the
# C3 bench line without the CPU leg; prints step time, shortlist average and the output digest.  Run from the repo
# root via gpurun.
set -eu
mkdir -p gpurun_out/pm
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for m in ${MODES:-0 3 4 5 0}; do
  TILER_ORBIT_PMODE=$m timeout -k 10 200 python3 -u bench.py --no-cpu --steps ${STEPS:-10} --no-keyframes --no-dither \
    --no-smooth --no-globaltiling --no-palettes ${EXTRA:-} > gpurun_out/pm/m$m.json 2> gpurun_out/pm/m$m.err
  python3 -c "import json; d=json.loads(open('gpurun_out/pm/m$m.json').read().strip().splitlines()[-1]); k=d['kernels']; print('pmode $m', d['ms_per_step'], k['nn_orbit']['ms_avg'], k['nn_rescore']['ms_avg'], k['nn_collect']['ms_avg'], d['search_stats'].get('fallback_queries'), d['out_digest'])"
done

#!/usr/bin/env bash
# C2: flat-tile grouping (one candidate split) vs none (the mixed split), experiment build, same box
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/fc2
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in flat noflat flat noflat; do
  if [ $v = noflat ]; then export TILER_NO_FLAT=1; else unset TILER_NO_FLAT; fi
  timeout -k 10 200 python3 -u bench.py --config c2 --no-cpu --steps 20 --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes > gpurun_out/fc2/$v.json 2> gpurun_out/fc2/$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/fc2/$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', d['ms_per_step'], k['nn_orbit']['ms_avg'], k['psyv']['ms_avg'], d['search_stats']['splits'], d['out_digest'])"
done

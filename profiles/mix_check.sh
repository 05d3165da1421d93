#!/usr/bin/env bash
# mixed candidate split (orbit_search): C2 bench with the CPU parity leg (front + back of the keyframe), then
# the experiment build with and without the mixed split (TILER_NO_MIX): identical output digests, shortlist time
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/mix
timeout -k 10 300 python3 bench.py --config c2 --steps 10 --no-keyframes --no-dither --no-globaltiling --no-palettes --no-smooth --cpu-seconds 15 > gpurun_out/mix/c2.json 2> gpurun_out/mix/c2.err
python3 -c "import json; d=json.loads(open('gpurun_out/mix/c2.json').read().strip().splitlines()[-1]); k=d['kernels']; c=d['cpu_baseline']; print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], k['nn_orbit']['ms_avg'], d['out_digest'], c['parity_queries'], c['parity_mismatches_vs_gpu'], c['dist_mismatches_vs_gpu'], c['sample'][:60])"
cp tiler_amd/lib/libANN.so /tmp/libANN_prod.so
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in mix nomix mix nomix; do
  if [ $v = nomix ]; then export TILER_NO_MIX=1; else unset TILER_NO_MIX; fi
  timeout -k 10 200 python3 -u bench.py --config c2 --no-cpu --steps 10 --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes > gpurun_out/mix/$v.json 2> gpurun_out/mix/$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/mix/$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', d['ms_per_step'], k['nn_orbit']['ms_avg'], k['nn_rescore']['ms_avg'], d['roofline']['frac'], d['out_digest'])"
done
cp /tmp/libANN_prod.so tiler_amd/lib/libANN.so

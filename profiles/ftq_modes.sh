#!/usr/bin/env bash
# Timing attribution of the fused FrameTiling query kernel (TILER_FTQ_MODE, experiment build only; results
# invalid in modes 1-2): 0 full, 1 without the Haar, 2 without the orbit transform.  Run from the repo root via
# gpurun; prints the kernel's average time per mode.
set -eu
mkdir -p gpurun_out/ftq
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for m in ${MODES:-0 2 3 5}; do
  TILER_FTQ_MODE=$m timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 --no-keyframes --no-dither --no-smooth \
    --no-globaltiling --no-palettes > gpurun_out/ftq/m$m.json 2> gpurun_out/ftq/m$m.err
  python3 -c "import json; d=json.loads(open('gpurun_out/ftq/m$m.json').read().strip().splitlines()[-1]); print('mode $m', d['kernels']['psyv']['ms_avg'], d['kernels']['nn_orbit']['ms_avg'])"
done

#!/usr/bin/env bash
# wave-parallel kd subtree kernel: kd / FrameTiling parity tests, then prepare timing new vs old (experiment build)
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/kd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_orbit.py tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/kd/tests.log 2>&1
echo "tests ok"
cp tiler_amd/lib/libANN.so /tmp/libANN_prod.so
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in new old; do
  if [ $v = old ]; then export TILER_KD_SUB_OLD=1; else unset TILER_KD_SUB_OLD; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 3 --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes > gpurun_out/kd/$v.json 2> gpurun_out/kd/$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/kd/$v.json').read().strip().splitlines()[-1]); p=d['secondary']['prepare']; print('$v', d['ms_per_step'], p['ms_each'], p['kd_build_ms_each'], d['out_digest'])"
done
cp /tmp/libANN_prod.so tiler_amd/lib/libANN.so

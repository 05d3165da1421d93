#!/usr/bin/env bash
# flat query tiles last: FrameTiling parity tests (incl. the large-batch vs per-frame check), the C3 bench with its
# CPU parity leg, then the experiment build with and without the flat reordering (TILER_NO_FLAT)
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/flat
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_frame_tiling.py tests/test_gpu_orbit.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/flat/tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python3 bench.py --steps 10 --no-keyframes --no-dither --no-globaltiling --no-palettes --no-smooth > gpurun_out/flat/bench_c3.json 2> gpurun_out/flat/bench_c3.err
python3 -c "import json; d=json.loads(open('gpurun_out/flat/bench_c3.json').read().strip().splitlines()[-1]); k=d['kernels']; print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], k['nn_orbit']['ms_avg'], d['out_digest'], d['cpu_baseline']['parity_mismatches_vs_gpu'], d['search_stats']['fallback_queries'])"
cp tiler_amd/lib/libANN.so /tmp/libANN_prod.so
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for v in flat noflat; do
  if [ $v = noflat ]; then export TILER_NO_FLAT=1; else unset TILER_NO_FLAT; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 10 --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes > gpurun_out/flat/$v.json 2> gpurun_out/flat/$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/flat/$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', d['ms_per_step'], k['nn_orbit']['ms_avg'], k['psyv']['ms_avg'], d['out_digest'])"
done
cp /tmp/libANN_prod.so tiler_amd/lib/libANN.so

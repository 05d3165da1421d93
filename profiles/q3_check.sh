#!/usr/bin/env bash
# fused query kernel with the fully unrolled transform: FrameTiling parity tests + C3 bench (digest, kernel times)
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/q3
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_frame_tiling.py tests/test_gpu_orbit.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/q3/tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python3 bench.py --steps 10 --no-keyframes --no-dither --no-globaltiling --no-palettes --no-smooth > gpurun_out/q3/bench_c3.json 2> gpurun_out/q3/bench_c3.err
python3 -c "import json; d=json.loads(open('gpurun_out/q3/bench_c3.json').read().strip().splitlines()[-1]); k=d['kernels']; print(d['value'], d['ms_per_step'], k['nn_orbit']['ms_avg'], k['psyv']['ms_avg'], k['psyv']['hbm_frac'], k['nn_collect']['ms_avg'], d['out_digest'], d['cpu_baseline']['parity_mismatches_vs_gpu'])"

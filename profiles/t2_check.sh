#!/usr/bin/env bash
# orbit tier-2 collect: FrameTiling / orbit / edge parity tests, then the C3 bench with its CPU parity leg
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/t2
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_orbit.py tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t2/tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python3 bench.py --steps 10 --no-keyframes --no-dither --no-globaltiling --no-palettes --no-smooth > gpurun_out/t2/bench_c3.json 2> gpurun_out/t2/bench_c3.err
python3 -c "import json; d=json.loads(open('gpurun_out/t2/bench_c3.json').read().strip().splitlines()[-1]); k=d['kernels']; print(d['value'], d['ms_per_step'], k['nn_orbit']['ms_avg'], k['nn_collect']['ms_avg'], k['nn_rescore2']['ms_avg'], k['nn_exact']['ms_avg'], d['search_stats'].get('fallback_queries'), d['search_stats'].get('exhaustive_queries'), d['out_digest'], d['cpu_baseline']['parity_mismatches_vs_gpu'])"

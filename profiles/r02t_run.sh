#!/usr/bin/env bash
# r02t: smooth tests, C3 bench (with the CPU leg), then the rocprofv3 trace + PMC passes (profiles/run_profile.sh)
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r02t
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_smooth.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r02t/smooth_tests.log 2>&1
echo "smooth tests done"
timeout -k 10 300 python3 bench.py --steps 10 --no-keyframes --no-dither --no-globaltiling --no-palettes > gpurun_out/r02t/bench_c3.json 2> gpurun_out/r02t/bench_c3.err
echo "bench done"
STEPS=2 bash profiles/run_profile.sh r02t

#!/usr/bin/env bash
# round-2 final profile set: Smooth parity tests, the C3 bench line (the driver's default flags), then
# the rocprofv3 trace + PMC passes of profiles/run_profile.sh
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/${TAG:-r02f}
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_smooth.py tests/test_pipeline.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG:-r02f}/smooth_tests.log 2>&1
echo "smooth tests done"
timeout -k 10 400 python3 bench.py --steps 10 > gpurun_out/${TAG:-r02f}/bench_c3.json 2> gpurun_out/${TAG:-r02f}/bench_c3.err
echo "bench done"
STEPS=2 bash profiles/run_profile.sh ${TAG:-r02f}

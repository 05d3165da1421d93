#!/usr/bin/env bash
# r02v: psyv / Smooth / pipeline parity tests (lane-per-item DCT kernel), the smooth probe, then the mixed-split A/B
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r02v
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_smooth.py tests/test_gpu_frame_tiling.py tests/test_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02v/tests.log 2>&1
echo "tests ok"
timeout -k 10 120 python3 tools/smooth_probe.py 5 > gpurun_out/r02v/smooth_probe.log 2>&1
tail -2 gpurun_out/r02v/smooth_probe.log
bash profiles/mix_check.sh

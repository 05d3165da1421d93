#!/usr/bin/env bash
# Round-3 targeted GPU pass: the search-path parity tests (incl. the full-size batch / tier-2 flood tests), then a
# C3 bench line.  Every GPU step has its own limit; the first failure ends the script (set -e).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03a}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_orbit.py tests/test_gpu_edges.py tests/test_gpu_frame_tiling.py tests/test_gpu_scale.py} -m gpu -x -v -s --timeout 900 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 300 python3 bench.py --steps 10 ${BENCH_ARGS:---no-keyframes --no-dither --no-palettes --no-globaltiling} > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"

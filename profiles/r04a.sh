#!/usr/bin/env bash
# Round 4, first pass: the new GPU tests (concurrent single-query callers on one handle, non-finite kd build), then the
# default bench line with the new secondary lines (per-tile calls, the 1000-frame encoder clips).  Every GPU step has
# its own limit; set -e ends the script at the first failure.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04a}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_concurrent.py tests/test_gpu_edges.py tests/test_gpu_frame_tiling.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"

#!/usr/bin/env bash
# Round 4 pass f: the small-batch exact scan (nn_scan_small_kernel) and the insertion-gated generic shortlist:
# the NN / FrameTiling / concurrency / edge GPU tests, then the default bench line.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04f
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_concurrent.py tests/test_gpu_edges.py tests/test_gpu_frame_tiling.py tests/test_gpu_orbit.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
echo "gpu tests done"; tail -2 "$OUT/gpu_tests.log"
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"

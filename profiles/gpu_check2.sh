#!/usr/bin/env bash
# One GPU pass for a kernel change (run from the repo root via gpurun): the FrameTiling / palette parity tests
# and a C3 bench line with the palette-generation secondary.
set -eu
TAG=${1:-check2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_orbit.py tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py \
  tests/test_gpu_palette.py tests/test_pipeline.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 bench.py --steps 10 --no-keyframes --no-dither --no-globaltiling > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench done"

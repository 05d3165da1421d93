#!/usr/bin/env bash
# r06: Yliluoma dither branch: dither GPU tests (incl. the refactored Thomas Knoll kernel), then the bench's dither line
set -eu
OUT=gpurun_out/${1:-r06y}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dither.py \
  tests/test_gpu_palette.py tests/test_pipeline.py > "$OUT/tests.log" 2>&1
echo "tests done"
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --no-smooth --no-keyframes --no-palettes --no-globaltiling \
  --no-encoder --no-per-call > "$OUT/bench_dither.json" 2> "$OUT/bench_dither.err"
echo "bench done"

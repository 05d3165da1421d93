#!/usr/bin/env bash
# r06: the query-half split with per-launch timers: orbit GPU tests, C3 / C5 bench lines, kernel trace of the C3 step
set -eu
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06sp}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_orbit.py tests/test_gpu_list_ties.py tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py > "$OUT/tests.log" 2>&1
echo "tests done"
timeout -k 10 400 python3 bench.py --steps 10 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "c3 done"
timeout -k 10 400 python3 bench.py --config c5 --steps 3 --no-keyframes --no-dither --no-palettes --no-globaltiling --cpu-seconds 20 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
echo "c5 done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-smooth --no-palettes --no-globaltiling --no-keyframes --no-dither --no-encoder --no-per-call > "$OUT/trace.log" 2>&1
echo "trace done"

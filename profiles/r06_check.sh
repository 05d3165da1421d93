#!/usr/bin/env bash
# r06: the tie reproducer, then the GPU tests touched by the list-insertion change (each step time-limited).
set -eu
OUT=gpurun_out/${1:-r06b}
mkdir -p "$OUT"
bash tools/merge_tie_repro.sh run > "$OUT/tie_repro.txt" 2>&1
echo "repro done"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_list_ties.py tests/test_gpu_scan_small.py tests/test_gpu_multidevice.py tests/test_gpu_concurrent.py \
  tests/test_gpu_frame_tiling.py > "$OUT/tests.log" 2>&1
echo "tests done"

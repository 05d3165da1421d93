#!/usr/bin/env bash
# r06: the k = 1 insertion gate of the generic shortlist: A/B on the shot-local and whole-tileset candidate sets, then
# the FrameTiling / edge / list-tie GPU tests (the gate is on by default)
set -eu
OUT=gpurun_out/${1:-r06h}
mkdir -p "$OUT"
for it in 16384 0; do
  for g in 1 0 1 0; do
    timeout -k 10 200 python3 -u tools/sl16_modes.py --item-tiles $it --gate $g --tag "items$it" >> "$OUT/ab.txt" 2>> "$OUT/ab.err"
  done
done
echo "ab done"
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py tests/test_gpu_list_ties.py tests/test_gpu_scale.py tests/test_gpu_orbit.py > "$OUT/tests.log" 2>&1
echo "tests done"

#!/usr/bin/env bash
# r06: shortlist in two query halves with the first half's rescore + pair pass on a second stream (A/B vs one launch),
# C3 step through tools/c3_step_probe.py (output digest), then the orbit GPU tests on the split build
set -eu
OUT=gpurun_out/${1:-r06z}
mkdir -p "$OUT"
for L in tools/_build/libANN_NS.so tiler_amd/lib/libANN.so tools/_build/libANN_NS.so tiler_amd/lib/libANN.so tools/_build/libANN_NS.so tiler_amd/lib/libANN.so; do
  timeout -k 10 200 python3 -u tools/c3_step_probe.py --lib $L --tag $(basename $L) --steps 20 >> "$OUT/ab.txt" 2>> "$OUT/ab.err"
done
echo "ab done"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_orbit.py tests/test_gpu_list_ties.py tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py tests/test_gpu_concurrent.py > "$OUT/tests.log" 2>&1
echo "tests done"

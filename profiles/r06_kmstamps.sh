#!/usr/bin/env bash
# r06: farthest-first round stamps (study build) + the GPU tests touched since r06c
set -eu
OUT=gpurun_out/${1:-r06d}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/ff_stamps.py --lib tools/_build/libANN_kmstamps.so > "$OUT/ff_stamps.json" 2> "$OUT/ff_stamps.err"
echo "stamps done"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_pipeline.py tests/test_gpu_multidevice.py tests/test_gpu_pri_search.py tests/test_gpu_kmodes.py > "$OUT/tests.log" 2>&1
echo "tests done"

#!/usr/bin/env bash
# r06: per-tile calls (16 native threads, one handle): callers spinning 200 / 0 / 50 us on their batch before sleeping
set -eu
OUT=gpurun_out/${1:-r06t}
mkdir -p "$OUT"
for L in tiler_amd/lib/libANN.so tools/_build/libANN_P0.so tools/_build/libANN_P50.so tiler_amd/lib/libANN.so tools/_build/libANN_P0.so tools/_build/libANN_P50.so; do
  timeout -k 10 200 python3 -u tools/percall_probe.py --lib $L --tag $(basename $L) >> "$OUT/percall.txt" 2>> "$OUT/percall.err"
done
echo "percall done"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_multidevice.py > "$OUT/tests.log" 2>&1
echo "tests done"

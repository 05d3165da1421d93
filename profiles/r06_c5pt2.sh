#!/usr/bin/env bash
# r06: per-handle coalescer slots (3 for scans of <= 96 MB of rows, else 2): C5 / C3 / plain per-tile calls + tests
set -eu
OUT=gpurun_out/${1:-r06x}
mkdir -p "$OUT"
timeout -k 10 200 python3 -u tools/c5_percall_ab.py tiler_amd/lib/libANN.so libANN.so >> "$OUT/c5.txt" 2>> "$OUT/c5.err"
timeout -k 10 200 python3 -u tools/percall_probe.py --tag libANN.so >> "$OUT/percall.txt" 2>> "$OUT/percall.err"
echo "probe done"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_concurrent.py tests/test_gpu_multidevice.py > "$OUT/tests.log" 2>&1
echo "tests done"

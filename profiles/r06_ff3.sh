#!/usr/bin/env bash
# r06: wave-item farthest-first: stamps (study build), K-Modes GPU tests, C4 GlobalTiling bench
set -eu
OUT=gpurun_out/${1:-r06e}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/ff_stamps.py --lib tools/_build/libANN_kmstamps.so > "$OUT/ff_stamps.json" 2> "$OUT/ff_stamps.err"
echo "stamps done"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kmodes.py tests/test_gpu_chain_c4.py tests/test_global_tiling.py > "$OUT/tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "gt done"

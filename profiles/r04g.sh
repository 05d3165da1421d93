#!/usr/bin/env bash
# Round 4 pass g: the C4 chain at size (tests/test_gpu_chain_c4.py).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04g
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_chain_c4.py -m gpu -x -v --timeout 850 --timeout-method thread --durations=5 > "$OUT/gpu_tests.log" 2>&1 || { tail -60 "$OUT/gpu_tests.log"; exit 1; }
tail -12 "$OUT/gpu_tests.log"

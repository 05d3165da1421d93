#!/usr/bin/env bash
# Round 5 pass w: UseOne's k = 8 preselection shortlist with one query block per wave (twice the waves) against the
# previous build (tools/k8_timing.py), k = 8 / palette-index / chain GPU tests, the new small-batch orbit FT test.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05w}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frame_tiling.py tests/test_gpu_chain_c4.py tests/test_gpu_concurrent.py tests/test_gpu_edges.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 120 python3 tools/k8_timing.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 120 python3 tools/k8_timing.py --tag new | tee -a "$OUT/ab.txt"
done

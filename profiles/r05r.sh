#!/usr/bin/env bash
# Round 5 pass r: the small-batch scan (per-tile calls) variants against the previous build (r2: scalar sums + pipelined
# A/B against the previous build: the per-call probe (scan kernel times at 1 / 4 / 16 queries, native 16-thread calls)
# and the k = 8 preselection kernel (tools/k8_timing.py; its 32x32x16 shortlist lost its packed seed ops too).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05r}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scan_small.py tests/test_gpu_concurrent.py tests/test_gpu_edges.py tests/test_gpu_frame_tiling.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python3 tools/percall_probe.py --tag new | tee -a "$OUT/ab.txt"
  timeout -k 10 120 python3 tools/k8_timing.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 120 python3 tools/k8_timing.py --tag new | tee -a "$OUT/ab.txt"
done

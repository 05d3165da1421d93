#!/usr/bin/env bash
# Round 5 pass p: partial-distance pruning in the small-batch scan (per-tile calls, k = 1).  Its tests and the
# per-call and kd-tree GPU tests, then the per-call line (bench.py's per_tile_calls, native harness) against the
# previous build.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05p}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scan_small.py tests/test_gpu_concurrent.py tests/test_gpu_edges.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python3 tools/percall_probe.py --tag new | tee -a "$OUT/ab.txt"
done

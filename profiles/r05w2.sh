#!/usr/bin/env bash
# Round 5 pass w2: the k = 1 small-batch scan of plain indexes from a row-interleaved copy (nn_scan_rows_kernel).
# NN / FT / orbit / per-call GPU tests, then the per-call probe against the previous commit's build (libANN_h.so):
# plain_262144 / plain_65536 / small_12000 are non-orbit handles (c3_262144 is a mirror-orbit index).  w3: only up
# to 65,536 candidates.  w4: the merge kernel replays in place and writes the results to host-visible memory
# (no replay launch, no copy back); libANN_h.so = the previous commit.  w9: the k = 1 merge in the wide form too.
# w10: the query row staged in LDS for the merge tail.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05w2}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scan_small.py tests/test_gpu_edges.py tests/test_gpu_orbit.py tests/test_gpu_concurrent.py tests/test_gpu_frame_tiling.py tests/test_gpu_pri_search.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_h.so --tag head | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python3 tools/percall_probe.py --tag new | tee -a "$OUT/ab.txt"
done

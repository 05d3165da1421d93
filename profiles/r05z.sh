#!/usr/bin/env bash
# Round 5 pass z: the small-batch scan on mirror-orbit indexes from the base rows only (nn_scan_orbit_kernel).  NN /
# FT / orbit / per-call GPU tests, then the per-call probe (C3 keyframe handle = an orbit index) against the previous
# build.  Pass z3: + the merge kernel (libANN_m); z4: libANN_m = the previous commit, new = + the group-order base copy; z5: one wave per (64-group block, query), base row in registers, compile-time mirror tables; z6: + XCD-aware order, every small batch.
# scan for groups of <= 4 queries).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05z}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scan_small.py tests/test_gpu_edges.py tests/test_gpu_orbit.py tests/test_gpu_concurrent.py tests/test_gpu_frame_tiling.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_m.so --tag head | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python3 tools/percall_probe.py --tag new | tee -a "$OUT/ab.txt"
done

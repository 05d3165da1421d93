#!/usr/bin/env bash
# Round 5 pass s: 16-byte loads in the index-build kernels (maxabs, prep_rows, prep16).  NN / FT / kd GPU tests, then
# ann_kdtree_create times against the previous build (tools/kd_build_probe.py create_ms) and the per-call probe.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05s}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kdtree_build.py tests/test_gpu_scan_small.py tests/test_gpu_edges.py tests/test_gpu_frame_tiling.py tests/test_gpu_orbit.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 200 python3 tools/kd_build_probe.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 200 python3 tools/kd_build_probe.py --tag new | tee -a "$OUT/ab.txt"
done

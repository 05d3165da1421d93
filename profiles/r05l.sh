#!/usr/bin/env bash
# Round 5 pass l: kd-tree build -- multi-wave subtree tops, wave-parallel quickselect, 128-point spread chunks folded
# per workgroup.  Build parity tests, then the build-time A/B against the previous build (tools/kd_build_probe.py).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05l}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kdtree_build.py tests/test_gpu_orbit.py tests/test_gpu_edges.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 200 python3 tools/kd_build_probe.py --lib tiler_amd/lib/ab/libANN_base.so --tag base | tee -a "$OUT/ab.txt"
  timeout -k 10 200 python3 tools/kd_build_probe.py --tag new | tee -a "$OUT/ab.txt"
done

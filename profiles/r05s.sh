#!/usr/bin/env bash
# Round 5 pass s (study): per-tile calls with 4 coalescer slots in flight per handle (libANN_x.so) against the
# shipped 2 (libANN_h.so = the build of the same commit); C3 keyframe handle, 16 native threads.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05s}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for i in 1 2; do
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_h.so --tag head | tee -a "$OUT/ab.txt"
  timeout -k 10 300 python3 tools/percall_probe.py --lib tiler_amd/lib/ab/libANN_x.so --tag new | tee -a "$OUT/ab.txt"
done

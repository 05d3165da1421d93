#!/usr/bin/env bash
# Round 5 pass y: the orbit shortlist with one query block per wave (12 or 16 waves per workgroup) against the shipped
# 8 waves x 2 query blocks, on bench.py's C3 step (tools/c3_step_probe.py), interleaved on one box.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05y}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for i in 1 2; do
  timeout -k 10 200 python3 tools/c3_step_probe.py --tag 8x2 | tee -a "$OUT/ab.txt"
  timeout -k 10 200 python3 tools/c3_step_probe.py --lib tiler_amd/lib/ab/libANN_orb_12x1.so --tag 12x1 | tee -a "$OUT/ab.txt"
  timeout -k 10 200 python3 tools/c3_step_probe.py --lib tiler_amd/lib/ab/libANN_orb_16x1.so --tag 16x1 | tee -a "$OUT/ab.txt"
done

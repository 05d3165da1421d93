#!/usr/bin/env bash
# Round 5 pass x: generic 16x16x32 shortlist shape A/B on a real PrepareFrameTiling candidate set (tools/sl16_modes.py):
# shipped 8 waves x 4 query blocks vs 16 x 2 and 12 x 3 (LDS holds one workgroup per CU, so waves per CU = NW).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05x}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for it in 16384 0; do
  for i in 1 2; do
    timeout -k 10 200 python3 tools/sl16_modes.py --item-tiles $it --tag "8x4 items=$it" | tee -a "$OUT/ab.txt"
    timeout -k 10 200 python3 tools/sl16_modes.py --item-tiles $it --lib tiler_amd/lib/ab/libANN_sl16_16x2.so --tag "16x2 items=$it" | tee -a "$OUT/ab.txt"
    timeout -k 10 200 python3 tools/sl16_modes.py --item-tiles $it --lib tiler_amd/lib/ab/libANN_sl16_12x3.so --tag "12x3 items=$it" | tee -a "$OUT/ab.txt"
  done
done

#!/usr/bin/env bash
# Round 5 pass g: UseOne's k = 8 preselection (tools/k8_timing.py, 16,384 items vs 262,144 64-d rows) with 4 (shipped),
# 2 and 1 waves per 32x32x16 shortlist workgroup (exp_push/libANN_nw*.so); digests must match.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05g}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so /tmp/libANN_nw4.so
for rep in 1 2; do
  for v in nw4 nw2 nw1; do
    if [ $v = nw4 ]; then cp /tmp/libANN_nw4.so tiler_amd/lib/libANN.so; else cp exp_push/libANN_$v.so tiler_amd/lib/libANN.so; fi
    timeout -k 10 120 python3 -u tools/k8_timing.py --tag "$v" >> "$OUT/k8.txt" 2>> "$OUT/k8.err"
    tail -1 "$OUT/k8.txt"
  done
done

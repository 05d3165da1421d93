#!/usr/bin/env bash
# Round 4 pass e (r04c.sh reused): VAR 5 = the insertion gate + the T-window lists; 0, 1 as before
# (tools/sl16_modes.py, experiment build, TILER_SL16_VAR: 1 per-query-block insertion gate with thresholds in
# registers, 2 three-buffer LDS ring, 3 both; 0 the shipped kernel).  Valid results: digests must match var 0.
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash profiles/exp_lib.sh
mkdir -p gpurun_out/r04e
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for it in 16384 0; do
  for v in 0 1 5 0 5; do
    TILER_SL16_VAR=$v timeout -k 10 120 python3 -u tools/sl16_modes.py --item-tiles $it --tag "it$it var$v" >> gpurun_out/r04e/var.txt 2>> gpurun_out/r04e/var.err
    tail -1 gpurun_out/r04e/var.txt
  done
done

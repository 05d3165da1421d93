#!/usr/bin/env bash
# Round 4 pass b: where the generic 16x16x32 shortlist's time goes on a real PrepareFrameTiling candidate set
# (tools/sl16_modes.py; experiment build, TILER_SL16_MODE: 1 no list insertion, 2 no epilogue, 3 = 2 without the
# A-fragment LDS reads inside a stage; 0 the shipped kernel).  Shot-local items (~100k candidates) then whole-tileset
# items (~388k).  Same box, one call; results of modes != 0 are invalid.
set -eu
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash profiles/exp_lib.sh
mkdir -p gpurun_out/r04b
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
for it in 16384 0; do
  for m in 0 1 2 3 0; do
    TILER_SL16_MODE=$m timeout -k 10 120 python3 -u tools/sl16_modes.py --item-tiles $it --tag it$it >> gpurun_out/r04b/modes.txt 2>> gpurun_out/r04b/modes.err
    tail -1 gpurun_out/r04b/modes.txt
  done
done

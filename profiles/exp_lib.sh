#!/usr/bin/env bash
# Build the timing-experiment library (tiler_amd/lib/experiments/libANN.so, make EXPERIMENTS=1) on the GPU box:
# it is listed in .gpurunignore, so no push carries it and the shipped tree never holds it.  Scripts that swap it in
# source this first.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ ! -f "$R/tiler_amd/lib/experiments/libANN.so" ]; then
  make -C "$R/tiler_amd/csrc" -j16 EXPERIMENTS=1 > /tmp/exp_lib_build.log 2>&1 || { tail -30 /tmp/exp_lib_build.log; exit 1; }
fi

#!/usr/bin/env bash
# Round 4 pass n: palette GPU tests on the shipped build, the DLv3 study dump, and the experiment build's phase split.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04n
mkdir -p "$OUT"
cd "$R"
bash "$R/profiles/exp_lib.sh"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_palette.py > "$OUT/pal_tests.log" 2>&1 || { tail -30 "$OUT/pal_tests.log"; exit 1; }
tail -1 "$OUT/pal_tests.log"
timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/ship.npz"
cp tiler_amd/lib/libANN.so /tmp/ship.so
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
TILER_DL3_PROF=1 timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/exp.npz" 2>&1 | grep -v kmeans_iter
cp /tmp/ship.so tiler_amd/lib/libANN.so

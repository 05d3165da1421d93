#!/usr/bin/env bash
# Round 4 pass r: palette GPU tests (shipped build), DLv3 study dumps of the shipped build, the experiment build
# (phase split) and the probe variant (tiler_amd/lib/var/probe: make EXPERIMENTS=1 EXTRA=-DDL3_PROBE=1).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04r
mkdir -p "$OUT"
cd "$R"
bash "$R/profiles/exp_lib.sh"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_palette.py > "$OUT/pal_tests.log" 2>&1 || { tail -30 "$OUT/pal_tests.log"; exit 1; }
tail -1 "$OUT/pal_tests.log"
timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/ship.npz"
cp tiler_amd/lib/libANN.so /tmp/ship.so
for v in experiments var/probe; do
  cp "tiler_amd/lib/$v/libANN.so" tiler_amd/lib/libANN.so
  echo "== $v"
  TILER_DL3_PROF=1 timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/$(basename $v).npz" 2>&1 | grep -v kmeans_iter
done
cp /tmp/ship.so tiler_amd/lib/libANN.so

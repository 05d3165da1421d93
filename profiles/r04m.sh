#!/usr/bin/env bash
# Round 4 pass m: palette GPU tests on the shipped build, then the DLv3 study dump (phase split of the largest pair)
# with the experiment build and three unroll-depth variants (tiler_amd/lib/var/u<U>m<UM>, built with
# make EXPERIMENTS=1 EXTRA="-DDL3_U_V=.. -DDL3_UM_V=..").
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04m
mkdir -p "$OUT"
cd "$R"
bash "$R/profiles/exp_lib.sh"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_palette.py > "$OUT/pal_tests.log" 2>&1 || { tail -30 "$OUT/pal_tests.log"; exit 1; }
tail -1 "$OUT/pal_tests.log"
timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/ship.npz"
cp tiler_amd/lib/libANN.so /tmp/ship.so
for v in experiments var/u8m4 var/u6m8 var/u10m4; do
  cp "tiler_amd/lib/$v/libANN.so" tiler_amd/lib/libANN.so
  echo "== $v"
  TILER_DL3_PROF=1 timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/$(basename $v).npz" 2>&1 | grep -v kmeans_iter
done
cp /tmp/ship.so tiler_amd/lib/libANN.so

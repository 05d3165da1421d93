#!/usr/bin/env bash
# Round 4 pass w: DLv3 unroll depths after the probe / immediate-offset changes (tiler_amd/lib/var/u<U>m<UM>,
# make EXTRA="-DDL3_U_V=.. -DDL3_UM_V=.."; shipped U 6, UM 4): tools/dl3_study.py dump times, palettes compared.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04w
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so /tmp/ship.so
for v in ship u6m8 u8m4 u8m8 ship; do
  if [ $v = ship ]; then cp /tmp/ship.so tiler_amd/lib/libANN.so; else cp tiler_amd/lib/var/$v/libANN.so tiler_amd/lib/libANN.so; fi
  echo "== $v"
  timeout -k 10 120 python3 -u tools/dl3_study.py dump "$OUT/$v.npz" | grep -v kmeans_iter
done
cp /tmp/ship.so tiler_amd/lib/libANN.so

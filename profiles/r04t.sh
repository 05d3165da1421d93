#!/usr/bin/env bash
# Round 4 pass t: tier-2 collect split count A/B (ORB_T2_WG builds in tiler_amd/lib/var/t2_*; shipped = 512 splits)
# at C3 and C2: the bench's nn_collect average and the step, same box; the digests must match.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04t
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so /tmp/ship.so
for cfg in c3 c2; do
  for v in ship t2_2048 t2_1024 t2_4096 ship; do
    if [ $v = ship ]; then cp /tmp/ship.so tiler_amd/lib/libANN.so; else cp tiler_amd/lib/var/$v/libANN.so tiler_amd/lib/libANN.so; fi
    timeout -k 10 200 python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu --no-smooth --no-palettes --no-globaltiling --no-encoder --no-per-call > "$OUT/$cfg.$v.json" 2> "$OUT/$cfg.$v.err"
    python3 -c "import json,sys;d=json.load(open('$OUT/$cfg.$v.json'));k=d['kernels'];print('$cfg','$v',d['value'],d['ms_per_step'],k['nn_collect']['ms_avg'],d.get('out_digest'))"
  done
done
cp /tmp/ship.so tiler_amd/lib/libANN.so

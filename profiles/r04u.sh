#!/usr/bin/env bash
# Round 4 pass u: the tier-2 split default (~1,024 workgroups, 128..512 splits) against the old fixed 512 splits
# (tiler_amd/lib/var/t2_0: make EXTRA=-DORB_T2_WG=0) at C3, C2 and C5: nn_collect average, step, digest.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04u
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so /tmp/ship.so
for cfg in c3 c2 c5; do
  for v in ship t2_0 ship; do
    if [ $v = ship ]; then cp /tmp/ship.so tiler_amd/lib/libANN.so; else cp tiler_amd/lib/var/$v/libANN.so tiler_amd/lib/libANN.so; fi
    timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu --no-smooth --no-palettes --no-globaltiling --no-encoder --no-per-call > "$OUT/$cfg.$v.json" 2> "$OUT/$cfg.$v.err"
    python3 -c "import json;d=json.load(open('$OUT/$cfg.$v.json'));k=d['kernels'];print('$cfg','$v',d['value'],d['ms_per_step'],k['nn_collect']['ms_avg'],d.get('out_digest'))"
  done
done
cp /tmp/ship.so tiler_amd/lib/libANN.so

#!/usr/bin/env bash
# Fused query kernel output stores, nt (1, default) vs sc1 (2: the lines leave L2 once written) vs plain (0), in the
# experiment build: C3 step and query-kernel time, then one FETCH_SIZE pass per mode (HBM reads per launch against the
# 199 MB of tile RGB).  Run from the repo root via gpurun; restores the shipped library at the end.
set -eu
R=$(pwd)
OUT=$R/gpurun_out/${1:-sc1}
mkdir -p "$OUT"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
B="bench.py --no-cpu --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes"
for v in 1 2 0 2 1; do
  TILER_FTQ_NT=$v timeout -k 10 200 python3 -u $R/$B --steps 10 > $OUT/b$v.json 2> $OUT/b$v.err
  python3 -c "import json; d=json.loads(open('$OUT/b$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('store mode $v', d['ms_per_step'], k['psyv']['ms_avg'], k['nn_orbit']['ms_avg'], d['out_digest'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 1 2; do
  TILER_FTQ_NT=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/p$v -o run --output-format csv -- python3 $R/$B --steps 2 --warmup 1 > $OUT/p$v.log 2>&1
  python3 - <<PY
import csv, glob
f = glob.glob("$OUT/p$v/**/run_counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "orbit_ft_query2" in r["Kernel_Name"]]
print("store mode $v FETCH_SIZE per launch (KiB units -> MB):", round(sum(v) / len(v) * 1024 / 1e6, 1), "launches", len(v))
PY
done
cd $R
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so

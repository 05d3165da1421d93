#!/usr/bin/env bash
# Fused query kernel, plain vs non-temporal output stores (experiment build, TILER_FTQ_NT=0/1): C3 bench step time
# and the query kernel's average, then one FETCH_SIZE / WRITE_SIZE pass each (HBM bytes per launch).  Also the
# tier-2 grid variants (t2grid_ab.sh).  Run from the repo root via gpurun.
set -eu
R=$(pwd)
mkdir -p gpurun_out/nt
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
B="bench.py --no-cpu --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes"
for v in 0 1 0 1; do
  TILER_FTQ_NT=$v timeout -k 10 200 python3 -u $B --steps 10 > gpurun_out/nt/b$v.json 2> gpurun_out/nt/b$v.err
  python3 -c "import json; d=json.loads(open('gpurun_out/nt/b$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('NT $v', d['ms_per_step'], k['psyv']['ms_avg'], k['nn_orbit']['ms_avg'], d['out_digest'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    TILER_FTQ_NT=$v timeout -s KILL 120 rocprofv3 --pmc $c -d $R/gpurun_out/nt/p$v$c -o run --output-format csv -- python3 $R/$B --steps 2 --warmup 1 > $R/gpurun_out/nt/p$v$c.log 2>&1
    python3 - <<PY
import csv, glob
f = glob.glob("$R/gpurun_out/nt/p$v$c/**/run_counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "orbit_ft_query2" in r["Kernel_Name"]]
print("NT $v $c per launch (KiB units -> MB):", round(sum(v) / len(v) * 1024 / 1e6, 1), "launches", len(v))
PY
  done
done
cd $R
bash profiles/t2grid_ab.sh

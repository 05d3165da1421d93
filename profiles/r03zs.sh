#!/usr/bin/env bash
# Round-3 pass zs: C2 and C5 FrameTiling lines on the final build (CPU parity sample on, secondaries off).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zs
mkdir -p "$OUT"
cd "$R"
F="--no-smooth --no-keyframes --no-dither --no-globaltiling --no-palettes"
for c in c2 c5; do
  timeout -k 10 400 python3 -u bench.py --config $c $F > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  python3 -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'].get('parity_mismatches_vs_gpu'), d['cpu_baseline'].get('parity_queries'))"
done

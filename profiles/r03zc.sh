#!/usr/bin/env bash
# Round-3 pass zc: the other BASELINE sizes on this round's build -- C2 (720p, 16k tileset x 4) and C5 (4K, 256k tileset
# x 4) bench lines with their CPU parity samples (no secondary lines).  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zc
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 bench.py --config c2 --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
python3 -c "import json; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'].get('parity_mismatches_vs_gpu'), d['cpu_baseline'].get('parity_queries'))"
timeout -k 10 500 python3 bench.py --config c5 --no-keyframes --no-dither --no-smooth --no-globaltiling --no-palettes > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
python3 -c "import json; d=json.loads(open('$OUT/bench_c5.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'].get('parity_mismatches_vs_gpu'), d['cpu_baseline'].get('parity_queries'))"

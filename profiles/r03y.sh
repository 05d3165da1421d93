#!/usr/bin/env bash
# Round-3 pass y: the sustained keyframe loop (bench_encoder.py, 1000-frame C3 clip, Medium quality) with shot-local
# items and with whole-tileset items, after the PrepareGlobalFT row-table fix.  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03y
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u bench_encoder.py --item-tiles 16384 > "$OUT/enc_local.json" 2> "$OUT/enc_local.err"
python3 -c "import json; d=json.loads(open('$OUT/enc_local.json').read().strip().splitlines()[-1]); print('local', d['value'], d['prepare_global_ms'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['wall_s'], d['parity'])"
timeout -k 10 400 python3 -u bench_encoder.py --check-kf -1 > "$OUT/enc_all.json" 2> "$OUT/enc_all.err"
python3 -c "import json; d=json.loads(open('$OUT/enc_all.json').read().strip().splitlines()[-1]); print('all', d['value'], d['prepare_global_ms'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['wall_s'])"

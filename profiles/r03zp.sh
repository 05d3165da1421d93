#!/usr/bin/env bash
# Round-3 pass zp: the shipped build after r03zo (farthest-first kmb_ff_persist2): K-Modes / GlobalTiling / pipeline
# GPU tests, the C4 GlobalTiling line with its CPU baseline (bins checked bit-exact), smoke.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zp
mkdir -p "$OUT"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 500 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
python3 -c "import json; d=json.loads(open('$OUT/gt.json').read().strip().splitlines()[-1]); print('gt', d['value'], d['digest'], d['phases'], d['cpu_baseline']['bins_mismatching_gpu'])"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"

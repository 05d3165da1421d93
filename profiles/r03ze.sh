#!/usr/bin/env bash
# Round-3 pass ze: K-Modes with the block-parallel ordered move list -- the K-Modes GPU tests (incl. K = 8,500 beyond
# the clash table, other modalities), the GlobalTiling / pipeline tests, the C4 line; then the other BASELINE sizes
# on this build: C2 (720p, 16k tileset x 4) and C5 (4K, 256k tileset x 4) bench lines with their CPU parity samples.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03ze
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kmodes.py tests/test_global_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/kmodes_tests.log" 2>&1
tail -1 "$OUT/kmodes_tests.log"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
python3 -c "import json; d=json.loads(open('$OUT/gt.json').read().strip().splitlines()[-1]); print('gt', d['value'], d['phases'], d['cpu_baseline']['bins_mismatching_gpu'])"
bash profiles/r03zc.sh
cp gpurun_out/r03zc/* "$OUT/"

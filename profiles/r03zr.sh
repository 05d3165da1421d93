#!/usr/bin/env bash
# Round-3 pass zr: the pair pass with rows staged through LDS in column chunks (experiment build, TILER_PAIRS_LDS=1)
# vs the per-lane row walk; C3 bench (no CPU, no secondaries), out_digest must not change; then the FrameTiling GPU
# tests on the variant.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03zr
mkdir -p "$OUT"
cd "$R"
cp tiler_amd/lib/libANN.so "$OUT/libANN.shipped.so"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
F="--no-cpu --no-smooth --no-keyframes --no-dither --no-globaltiling --no-palettes --steps 10"
for v in 0 1 0 1; do
  TILER_PAIRS_LDS=$v timeout -k 10 200 python3 -u bench.py $F > "$OUT/b$v.json" 2> "$OUT/b$v.err"
  python3 -c "import json; d=json.loads(open('$OUT/b$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('LDS $v', d['value'], d['out_digest'], 'pairs', k['nn_pairs']['ms_avg'], 'rescore', k['nn_rescore']['ms_avg'], 'orbit', k['nn_orbit']['ms_avg'])"
done
TILER_PAIRS_LDS=1 timeout -k 10 500 python3 -u -m pytest tests -m gpu -k "frame_tiling or orbit or pipeline or c3 or c5" -x -v --timeout 400 --timeout-method thread > "$OUT/tests_lds.log" 2>&1
tail -1 "$OUT/tests_lds.log"
cp "$OUT/libANN.shipped.so" tiler_amd/lib/libANN.so
rm -f "$OUT/libANN.shipped.so"

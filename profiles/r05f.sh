#!/usr/bin/env bash
# Round 5 pass f: per-call path with the wave-parallel fused pruning check (concurrency / edge / frame-tiling GPU tests,
# bench per-call line), then the generic shortlist A/B: VAR 1 (shipped, CB 8), 8 (CB 4, same insertion), 9 (CB 4 +
# insertions queued per lane in LDS) -- tools/sl16_modes.py, experiment build pushed in exp_push/.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05f}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_concurrent.py tests/test_gpu_edges.py tests/test_gpu_frame_tiling.py \
  tests/test_gpu_multidevice.py -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -80 "$OUT/gpu_tests.log"; exit 1; }
echo "gpu tests done"; tail -1 "$OUT/gpu_tests.log"; grep "calls/s" "$OUT/gpu_tests.log" || true
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-smooth --no-keyframes --no-dither --no-palettes \
  --no-globaltiling --no-encoder > "$OUT/bench_percall.json" 2> "$OUT/bench_percall.err"
python3 -c "import json; d=json.load(open('$OUT/bench_percall.json')); print(json.dumps(d['secondary']['per_tile_calls']))"
cp exp_push/libANN.so tiler_amd/lib/libANN.so
for it in 16384 0; do
  for v in 1 9 8 1 9; do
    TILER_SL16_VAR=$v timeout -k 10 120 python3 -u tools/sl16_modes.py --item-tiles $it --tag "it$it var$v" >> "$OUT/sl16_var.txt" 2>> "$OUT/sl16_var.err"
    tail -1 "$OUT/sl16_var.txt"
  done
done

#!/usr/bin/env bash
# Round 5 pass d: the whole GPU suite on this build (fused small-batch pruning check, two in-flight coalesced batches,
# forced-replay test), the per-call line natively, and a kernel trace of the native per-call harness.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05d}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread --durations=15 > "$OUT/gpu_tests.log" 2>&1 || { tail -80 "$OUT/gpu_tests.log"; exit 1; }
echo "gpu tests done"; tail -1 "$OUT/gpu_tests.log"; grep "calls/s" "$OUT/gpu_tests.log" || true
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-smooth --no-keyframes --no-dither --no-palettes \
  --no-globaltiling --no-encoder > "$OUT/bench_percall.json" 2> "$OUT/bench_percall.err"
python3 -c "import json; d=json.load(open('$OUT/bench_percall.json')); print(json.dumps(d['secondary']['per_tile_calls']))"

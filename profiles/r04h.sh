#!/usr/bin/env bash
# Round 4 pass h: the whole GPU suite on this build, smoke, the default bench line, the C4 GlobalTiling line.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04h}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > "$OUT/gpu_tests.log" 2>&1 || { tail -60 "$OUT/gpu_tests.log"; exit 1; }
echo "gpu tests done"; tail -3 "$OUT/gpu_tests.log"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"

#!/usr/bin/env bash
# One GPU-box pass (run through gpurun from the repo root): GPU parity suite -> smoke() -> bench lines at C3, C2, C5.
# Every GPU step has its own time limit; the first failure ends the script (set -e).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-check}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  echo "gpu tests done"
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  echo "smoke done"
fi
timeout -k 10 300 python3 bench.py --steps 10 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"
if [ "${MORE:-1}" = "1" ]; then
  timeout -k 10 300 python3 bench.py --config c2 --steps 10 --no-keyframes --no-dither --no-palettes --no-globaltiling > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
  echo "bench c2 done"
  timeout -k 10 400 python3 bench.py --config c5 --steps 3 --no-keyframes --no-dither --no-palettes --no-globaltiling --cpu-seconds 20 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
  echo "bench c5 done"
fi

#!/usr/bin/env bash
# Round-3 pass e: the whole GPU suite (incl. the full-size batch, C5 and tier-2 flood tests), smoke, then the
# default C3 bench line.  Every GPU step has its own limit; set -e ends the script at the first failure.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03e}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 840 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYARGS:-} > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 240 python3 bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"

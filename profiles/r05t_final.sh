#!/usr/bin/env bash
# Round 5 last check: the whole GPU suite and smoke on the final build.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05t_final
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"

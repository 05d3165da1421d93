#!/usr/bin/env bash
# r06: full GPU suite + smoke + default bench line (each step time-limited, stop at the first failure).
set -eu
OUT=gpurun_out/${1:-r06c}
mkdir -p "$OUT"
if [ "${PRE:-}" = tie ]; then
  bash tools/merge_tie_repro.sh detail > "$OUT/tie_repro_detail.txt" 2>&1
  timeout -k 10 300 python3 -u tools/oldmerge_check.py --lib tools/_build/libANN_r05oldmerge.so > "$OUT/oldmerge_check.txt" 2>&1
  echo "tie studies done"
fi
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 400 python3 bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench done"

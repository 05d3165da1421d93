#!/usr/bin/env bash
# r06: device-written K-Modes work list + quad-DPP pair pass: full GPU suite, smoke, C4 bench + kernel trace
set -eu
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06p}
mkdir -p "$OUT"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 300 python3 bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "gt done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o kt -- python3 "$R/bench_globaltiling.py" --no-cpu > "$OUT/gt_traced.json" 2> "$OUT/gt_traced.err"
echo "trace done"

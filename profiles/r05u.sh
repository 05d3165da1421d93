#!/usr/bin/env bash
# Round 5 pass u (and later final passes): the current build -- whole GPU suite, smoke, the default bench line
# (with the clip-level palette line), and the kernel trace of a short headline run.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05h}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > "$OUT/gpu_tests.log" 2>&1 || { tail -60 "$OUT/gpu_tests.log"; exit 1; }
echo "gpu tests done"; tail -1 "$OUT/gpu_tests.log"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-smooth --no-palettes --no-globaltiling --no-encoder --no-per-call --no-keyframes --no-dither > "$OUT/trace.log" 2>&1
echo "trace done"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/trace"

#!/usr/bin/env bash
# Round-3 final pass: the whole GPU suite, smoke, the default C3 bench line, the C4 GlobalTiling line, then the profile
# set of this build (rocprofv3 --kernel-trace --stats + separate PMC passes, profiles/run_profile.sh).  Every GPU step
# has its own limit; set -e ends the script at the first failure.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03end}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 500 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 240 python3 bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
echo "bench c3 done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "globaltiling done"
bash profiles/run_profile.sh $TAG/prof
echo "profile done"

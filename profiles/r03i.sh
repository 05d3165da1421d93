#!/usr/bin/env bash
# Round-3 pass i: the profile set of the current build (rocprofv3 --kernel-trace --stats + separate PMC passes of the
# C3 bench step, profiles/run_profile.sh), then a kernel trace of the C4 GlobalTiling run (per-dispatch durations of
# the K-Modes chain).  Each step has its own limit; set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03i}
cd "$R"
bash profiles/run_profile.sh $TAG
mkdir -p "$R/gpurun_out/$TAG/gt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/gt" -o run --output-format csv -- python3 $R/bench_globaltiling.py --no-cpu > "$R/gpurun_out/$TAG/gt/gt.log" 2>&1
echo "gt trace done"

#!/usr/bin/env bash
# Round-3 pass p: per-dispatch kernel trace of the C4 GlobalTiling run (K-Modes chain: where the sequential passes
# spend their 0.3 s), shipped build.  set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03p}
mkdir -p "$R/gpurun_out/$TAG/gt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG/gt" -o run --output-format csv -- python3 $R/bench_globaltiling.py --no-cpu > "$R/gpurun_out/$TAG/gt/gt.log" 2>&1
echo "gt trace done"

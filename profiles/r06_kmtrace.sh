#!/usr/bin/env bash
# r06: kernel trace of the C4 K-Modes call (per-iteration host bubbles, late-step launch timeline)
set -eu
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06kt}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o kt -- python3 "$R/bench_globaltiling.py" --no-cpu > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "trace done"

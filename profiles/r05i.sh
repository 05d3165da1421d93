#!/usr/bin/env bash
# Round 5 pass i: does keyframe k+1's Prepare run beside keyframe k's FrameTiling in the encoder loop?  Kernel +
# HIP API trace of a 240-frame clip (10 keyframes, shot-local items), analysed by tools/overlap_trace.py.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05i}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$OUT/trace" -o run --output-format csv -- python3 $R/bench_encoder.py --frames 240 --item-tiles 16384 --check-kf -1 > "$OUT/enc.json" 2> "$OUT/enc.err"
echo "trace done"
python3 $R/tools/overlap_trace.py "$OUT/trace" > "$OUT/overlap.txt" 2>&1
cat "$OUT/overlap.txt"
rm -rf "$OUT/trace"

#!/usr/bin/env bash
# r06: kernel trace + stats of the sustained encoder loop with items from the whole tileset (240 frames = 10 keyframes)
set -eu
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06ea}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o enc -- python3 "$R/bench_encoder.py" --frames 240 --check-kf -1 > "$OUT/enc.json" 2> "$OUT/enc.err"
echo "trace done"

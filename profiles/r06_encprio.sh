#!/usr/bin/env bash
# r06: the sustained encoder loop with the next keyframe's Prepare on a high-priority stream vs a normal one (one box)
set -eu
OUT=gpurun_out/${1:-r06k}
mkdir -p "$OUT"
for it in 16384 0; do
  for pr in 1 0 1 0; do
    timeout -k 10 300 python3 -u bench_encoder.py --item-tiles $it --prep-priority $pr --check-kf -1 > "$OUT/enc_${it}_${pr}.json" 2>> "$OUT/enc.err"
    python3 -c "import json,sys; d=json.loads(open('$OUT/enc_${it}_${pr}.json').read().strip().splitlines()[-1]); print('items', $it, 'prio', $pr, d['value'], d['wall_s'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['out_digest'])" >> "$OUT/summary.txt"
  done
done
echo "enc done"

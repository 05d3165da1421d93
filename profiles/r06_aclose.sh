#!/usr/bin/env bash
# r06: the encoder loop with the previous handle closed by a closer thread (--async-close 1) against closed on the
# launching thread (0): both item modes, alternating, same digests and keyframe re-check expected
set -eu
OUT=gpurun_out/${1:-r06ac}
mkdir -p "$OUT"
for it in 16384 0; do
  for PP in 0 1 0 1 0 1; do
    timeout -k 10 300 python3 -u bench_encoder.py --item-tiles $it --check-kf 1 --async-close $PP > "$OUT/enc.json" 2> "$OUT/enc_${it}_${PP}.err"
    python3 -c "import json; d=json.loads(open('$OUT/enc.json').read().strip().splitlines()[-1]); print('async-close', $PP, $it, d['value'], d['wall_s'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['loop_ms_avg'], d['out_digest'], d['parity']['mismatches_total'])" >> "$OUT/ab.txt"
  done
done
echo "ab done"

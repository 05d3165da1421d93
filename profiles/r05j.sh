#!/usr/bin/env bash
# Round 5 pass j (the --reserve-cus flag and tiler_stream_create_partition were removed after it): encoder loop with the next keyframe's Prepare on reserved CUs (tiler_stream_create_partition):
# A/B over the reserve on 240-frame clips (10 keyframes), shot-local and whole-tileset items.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05j}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for items in 16384 0; do
  for rc in 0 32 16 64 0 32; do
    timeout -k 10 200 python3 bench_encoder.py --frames 240 --item-tiles $items --check-kf -1 --reserve-cus $rc > "$OUT/enc_${items}_${rc}.json" 2> "$OUT/enc_${items}_${rc}.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['wall_s'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['out_digest'])" "$OUT/enc_${items}_${rc}.json" $items $rc | tee -a "$OUT/ab.txt"
  done
done

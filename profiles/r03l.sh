#!/usr/bin/env bash
# Round-3 pass l: K-Modes (persistent farthest-first with sc1 hand-offs: tests, C4 line, per-launch A/B), then the
# sustained keyframe loop after the 16-lane generic rescore: shot-local items with the CPU re-check of keyframe 1
# (heartbeat every 30 s), and whole-tileset items.  Each step has its own limit; set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03l}
OUT=$R/gpurun_out/$TAG
cd "$R"
bash profiles/r03k.sh $TAG
timeout -k 10 600 python3 -u bench_encoder.py --item-tiles 16384 > "$OUT/enc_local.json" 2> "$OUT/enc_local.err"
echo "encoder local (checked) done"
timeout -k 10 300 python3 -u bench_encoder.py --check-kf -1 > "$OUT/enc_all.json" 2> "$OUT/enc_all.err"
echo "encoder all done"

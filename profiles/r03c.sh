#!/usr/bin/env bash
# Round-3 pass c: sustained keyframe loop (overlapped, checked; and with shot-local items), then the experiment A/Bs.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03c
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -u bench_encoder.py > "$OUT/enc_ovl.json" 2> "$OUT/enc_ovl.err"
echo "encoder overlap done"
timeout -k 10 300 python3 -u bench_encoder.py --check-kf -1 --item-tiles 16384 > "$OUT/enc_ovl_local.json" 2> "$OUT/enc_ovl_local.err"
echo "encoder overlap local done"
timeout -k 10 300 python3 -u bench_encoder.py --check-kf -1 --item-tiles 16384 --no-overlap > "$OUT/enc_seq_local.json" 2> "$OUT/enc_seq_local.err"
echo "encoder seq local done"
bash profiles/ftq_nt_ab.sh > "$OUT/ab.log" 2>&1
echo "ab done"

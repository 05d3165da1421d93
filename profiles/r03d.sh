#!/usr/bin/env bash
# Round-3 pass d: sustained keyframe loop, C4 GlobalTiling with the cooperative K-Modes (then the per-launch form for
# A/B), then the experiment-build A/Bs.  Every step has its own limit; set -e ends the script at the first failure.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03d
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -u bench_encoder.py > "$OUT/enc_ovl.json" 2> "$OUT/enc_ovl.err"
echo "encoder overlap done"
timeout -k 10 300 python3 -u bench_encoder.py --check-kf -1 --item-tiles 16384 > "$OUT/enc_ovl_local.json" 2> "$OUT/enc_ovl_local.err"
echo "encoder overlap local done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt_coop.json" 2> "$OUT/gt_coop.err"
echo "globaltiling coop done"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
TILER_KM_COOP=0 timeout -k 10 300 python3 -u bench_globaltiling.py --no-cpu > "$OUT/gt_launch.json" 2> "$OUT/gt_launch.err"
echo "globaltiling per-launch done"
bash profiles/ftq_nt_ab.sh > "$OUT/ab.log" 2>&1
echo "ab done"

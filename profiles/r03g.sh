#!/usr/bin/env bash
# Round-3 pass g: sustained keyframe loop with diagnostics (no CPU re-check), C4 GlobalTiling, then the experiment A/Bs
# (query-kernel store modes; shortlist VALU spread, pmode 13).  Each GPU step has its own limit; set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03g}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u bench_encoder.py --check-kf -1 > "$OUT/enc_ovl.json" 2> "$OUT/enc_ovl.err"
echo "encoder done"
timeout -k 10 300 python3 -u bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "globaltiling done"
bash profiles/ftq_sc1_ab.sh $TAG/sc1 > "$OUT/sc1_ab.log" 2>&1
echo "sc1 ab done"
MODES="0 13 0 13" bash profiles/pmode_ab.sh > "$OUT/pmode_ab.log" 2>&1
echo "pmode ab done"

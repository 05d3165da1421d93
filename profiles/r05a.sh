#!/usr/bin/env bash
# Round 5 pass a: bench.py's own N-rank launch on the one-GPU box (gloo rehearsal, every rank on cuda:0), then the
# headline kernel's kernel trace + PMC passes on the round-5 build (refreshes profiles/pmc_traffic.json).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05a}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
TILER_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu \
  --no-smooth --no-keyframes --no-dither --no-palettes --no-globaltiling --no-encoder --no-per-call \
  > "$OUT/bench_n2_rehearsal.json" 2> "$OUT/bench_n2_rehearsal.err"
echo "n2 rehearsal done"; head -c 400 "$OUT/bench_n2_rehearsal.json"; echo
STEPS=3 bash profiles/run_profile.sh "$TAG"
python3 profiles/summarize.py "$OUT" "$OUT/pmc_traffic.json" > "$OUT/summary.json"
echo "summary done"

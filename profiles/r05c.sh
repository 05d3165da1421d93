#!/usr/bin/env bash
# Round 5 pass c (= r05b with the multidevice worker fixed) + the generic shortlist A/B: VAR 1 (shipped) vs VAR 5
# (software-pipelined stage, one compare per element; tools/sl16_modes.py, experiment build pushed in exp_push/).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05c}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multidevice.py tests/test_gpu_concurrent.py tests/test_gpu_edges.py \
  -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/gpu_tests_new.log" 2>&1 || { tail -80 "$OUT/gpu_tests_new.log"; exit 1; }
echo "new gpu tests done"; tail -3 "$OUT/gpu_tests_new.log"; grep "calls/s" "$OUT/gpu_tests_new.log" || true
TILER_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu \
  --no-smooth --no-keyframes --no-dither --no-palettes --no-globaltiling --no-encoder --no-per-call \
  > "$OUT/bench_n2_rehearsal.json" 2> "$OUT/bench_n2_rehearsal.err"
echo "n2 rehearsal done"; head -c 300 "$OUT/bench_n2_rehearsal.json"; echo
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-encoder --no-globaltiling --no-palettes \
  > "$OUT/bench_short.json" 2> "$OUT/bench_short.err"
echo "short bench done"
STEPS=3 bash profiles/run_profile.sh "$TAG"
python3 profiles/summarize.py "$OUT" "$OUT/pmc_traffic.json" > "$OUT/summary.json"
echo "summary done"
cp exp_push/libANN.so tiler_amd/lib/libANN.so
for it in 16384 0; do
  for v in 1 5 1 5; do
    TILER_SL16_VAR=$v timeout -k 10 120 python3 -u tools/sl16_modes.py --item-tiles $it --tag "it$it var$v" >> "$OUT/sl16_var.txt" 2>> "$OUT/sl16_var.err"
    tail -1 "$OUT/sl16_var.txt"
  done
done

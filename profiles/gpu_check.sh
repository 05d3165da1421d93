#!/usr/bin/env bash
# One GPU-box pass over the current build (run through gpurun from the repo root):
#   GPU parity suite -> smoke() -> default bench line -> rocprofv3 trace + PMC passes (run_profile.sh).
# Every GPU step has its own time limit; the first failure ends the script.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-check}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "gpu tests done"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke done"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench done"
if [ "${N2:-0}" = "1" ]; then
  # N>1 control flow rehearsed on the one-GPU box: 2 ranks on cuda:0 over gloo (the driver runs RCCL on 8 GPUs)
  TILER_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --no-cpu \
    > "$OUT/bench_n2_gloo.json" 2> "$OUT/bench_n2_gloo.err"
  echo "n2 rehearsal done"
fi
if [ "${PROFILE:-1}" = "1" ]; then
  bash "$R/profiles/run_profile.sh" "$TAG/prof"
fi

#!/usr/bin/env bash
# r06 final build: the N = 2 path rehearsed on the one-GPU box (both ranks on cuda:0, gloo: RCCL refuses two ranks
# on one device), bench.py spawning its own ranks; then N = 1 under a launcher on nccl (RCCL at world size 1)
set -eu
OUT=gpurun_out/${1:-r06n2}
mkdir -p "$OUT"
TILER_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu \
  --no-smooth --no-keyframes --no-dither --no-palettes --no-globaltiling --no-encoder --no-per-call \
  > "$OUT/bench_n2_gloo_rehearsal.json" 2> "$OUT/bench_n2_gloo_rehearsal.err"
echo "n2 done"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu --no-smooth --no-keyframes --no-dither --no-palettes --no-globaltiling \
  --no-encoder --no-per-call > "$OUT/bench_n1_launcher_nccl.json" 2> "$OUT/bench_n1_launcher_nccl.err"
echo "n1 launcher done"

#!/usr/bin/env bash
# Profile bench.py on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats  -> per-kernel durations (compare with bench.py's HIP-event timing)
#   2. separate --pmc passes (no trace domains mixed in): MFMA busy / clock, HBM FETCH_SIZE, WRITE_SIZE, LDS
# Outputs land in gpurun_out/$TAG/ ; copy the summaries to profiles/ afterwards.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
STEPS=${STEPS:-2}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps $STEPS --warmup 1 --no-cpu --no-smooth --no-palettes --no-globaltiling --no-keyframes --no-dither --no-encoder --no-per-call"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $BENCH > "$OUT/trace.log" 2>&1
echo "trace done"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  -d "$OUT/pmc_sq" -o run --output-format csv -- $BENCH > "$OUT/pmc_sq.log" 2>&1
echo "pmc sq done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- $BENCH > "$OUT/pmc_fetch.log" 2>&1
echo "pmc fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- $BENCH > "$OUT/pmc_write.log" 2>&1
echo "pmc write done"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU \
  -d "$OUT/pmc_inst" -o run --output-format csv -- $BENCH > "$OUT/pmc_inst.log" 2>&1
echo "pmc inst done"

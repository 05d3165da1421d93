#!/usr/bin/env bash
# Round 4 pass q: memory-side PMC counters of dl3_reduce_kernel (L2 hit rate, TCP->TCC read latency, VMEM read
# instructions and their issue cycles) on tools/dl3_study.py's workload.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04q
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
p=mem
timeout -s KILL 150 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr -d /tmp/r04q_${p} -o run --output-format csv -- python3 $R/tools/dl3_study.py dump /tmp/x.npz > "$OUT/$p.log" 2>&1 || { tail -20 "$OUT/$p.log"; exit 1; }
python3 $R/profiles/pmc_rows.py /tmp/r04q_${p} dl3_reduce > "$OUT/$p.csv"
rm -rf /tmp/r04q_${p}
cat "$OUT/$p.csv"

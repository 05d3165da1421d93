#!/usr/bin/env bash
# Round 4 pass o: PMC counters of dl3_reduce_kernel (DLv3 pass 2) on tools/dl3_study.py's workload: two passes,
# only the kernel's rows kept (profiles/pmc_rows.py).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04o
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for pass in "sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "inst SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  set -- $pass
  p=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d /tmp/r04o_${p} -o run --output-format csv -- python3 $R/tools/dl3_study.py dump /tmp/x.npz > "$OUT/$p.log" 2>&1 || { tail -20 "$OUT/$p.log"; exit 1; }
  python3 $R/profiles/pmc_rows.py /tmp/r04o_${p} dl3_reduce > "$OUT/$p.csv"
  rm -rf /tmp/r04o_${p}
  echo "$p done"; cat "$OUT/$p.csv"
done

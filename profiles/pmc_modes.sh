#!/usr/bin/env bash
# PMC comparison of the orbit shortlist's timing-experiment modes (TILER_ORBIT_MODE): co-execution of
# VALU and MFMA, LDS issue stalls.  Outputs gpurun_out/pmcm/<mode>/.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
for m in ${MODES:-0 2 3}; do
  TILER_ORBIT_MODE=$m timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d "$R/gpurun_out/pmcm/$m" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-smooth \
    > "$R/gpurun_out/pmcm/m$m.log" 2>&1
  echo "mode $m done"
done

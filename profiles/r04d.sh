#!/usr/bin/env bash
# Round 4 pass d: PMC counters of the generic 16x16x32 shortlist on the shot-local candidate set (tools/sl16_modes.py,
# one timed rep): shipped kernel, VAR 1, timing MODE 1 (no insertion) and MODE 3 (floor).  Two passes per config; only
# the shortlist's rows are kept (profiles/pmc_rows.py).
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04d
mkdir -p "$OUT"
cd "$R"
bash "$R/profiles/exp_lib.sh"
cp tiler_amd/lib/experiments/libANN.so tiler_amd/lib/libANN.so
cd /tmp
export TMPDIR=/tmp
for cfg in "v0 TILER_SL16_VAR=0" "v1 TILER_SL16_VAR=1" "m1 TILER_SL16_MODE=1" "m3 TILER_SL16_MODE=3"; do
  set -- $cfg
  name=$1
  export $2
  for pass in "sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
              "inst SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
    set -- $pass
    p=$1; shift
    timeout -k 10 200 rocprofv3 --pmc "$@" -d /tmp/r04d_${name}_${p} -o run --output-format csv -- python3 $R/tools/sl16_modes.py --reps 1 --tag $name > "$OUT/$name.$p.log" 2>&1 || { tail -20 "$OUT/$name.$p.log"; exit 1; }
    python3 $R/profiles/pmc_rows.py /tmp/r04d_${name}_${p} nn_shortlist16 > "$OUT/$name.$p.csv"
    rm -rf /tmp/r04d_${name}_${p}
  done
  unset TILER_SL16_VAR TILER_SL16_MODE
  echo "$name done"; cat "$OUT/$name.sq.csv" "$OUT/$name.inst.csv"
done

#!/bin/bash
# r03zj: C4 GlobalTiling K-Modes timed with the kernel timers off (after one untimed run); then a kernel trace of
# one K-Modes call for the per-step durations and gaps (assign / decide / apply)
set -o pipefail
OUT=gpurun_out/r03zj; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench_globaltiling.py --no-cpu > $OUT/gt.json 2> $OUT/gt.err && tail -1 $OUT/gt.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o kt -- python3 -u bench_globaltiling.py --no-cpu > $OUT/gt_traced.json 2> $OUT/gt_traced.err &&
python3 profiles/r03zj_steps.py $OUT/trace > $OUT/steps.txt && cat $OUT/steps.txt

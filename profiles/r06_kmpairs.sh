#!/usr/bin/env bash
# r06: K-Modes work list reused across iterations (tests, C4 bench, kernel trace) + the quad-DPP pair pass and rescore occupancy A/B (C3 step)
set -eu
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06o}
mkdir -p "$OUT"
for L in tiler_amd/lib/libANN.so tools/_build/libANN_Q.so tools/_build/libANN_R.so tools/_build/libANN_QR.so tiler_amd/lib/libANN.so tools/_build/libANN_Q.so tools/_build/libANN_R.so tools/_build/libANN_QR.so; do
  timeout -k 10 200 python3 -u tools/c3_step_probe.py --lib $L --tag $(basename $L) --steps 20 >> "$OUT/pairs_ab.txt" 2>> "$OUT/pairs_ab.err"
done
echo "pairs ab done"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kmodes.py tests/test_gpu_chain_c4.py tests/test_global_tiling.py > "$OUT/km_tests.log" 2>&1
echo "km tests done"
timeout -k 10 300 python3 bench_globaltiling.py > "$OUT/gt.json" 2> "$OUT/gt.err"
echo "gt done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o kt -- python3 "$R/bench_globaltiling.py" --no-cpu > "$OUT/gt_traced.json" 2> "$OUT/gt_traced.err"
echo "trace done"

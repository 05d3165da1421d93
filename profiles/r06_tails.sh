#!/usr/bin/env bash
# r06: occupancy variants of the orbit rescore / pair pass (C3 step, one box), then the scaling model
set -eu
OUT=gpurun_out/${1:-r06i}
mkdir -p "$OUT"
for L in tiler_amd/lib/libANN.so tools/_build/libANN_A.so tools/_build/libANN_B.so tools/_build/libANN_C.so tiler_amd/lib/libANN.so tools/_build/libANN_A.so tools/_build/libANN_C.so; do
  timeout -k 10 200 python3 -u tools/c3_step_probe.py --lib $L --tag $(basename $L) --steps 20 >> "$OUT/ab.txt" 2>> "$OUT/ab.err"
done
echo "ab done"
timeout -k 10 600 python3 -u tools/scaling_model.py --bench profiles/r06/c_bench_c3.json > "$OUT/scaling_model.json" 2> "$OUT/scaling_model.err"
echo "model done"

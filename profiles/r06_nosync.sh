#!/usr/bin/env bash
# r06: no device-wide wait when a handle's first search has no scratch to file back (the encoder's FrameTiling no
# longer waits for the next keyframe's Prepare): encoder loop A/B, both item modes, then the FrameTiling-side GPU tests
set -eu
OUT=gpurun_out/${1:-r06ns}
mkdir -p "$OUT"
for it in 0 16384; do
  for L in tools/_build/libANN_S0.so tiler_amd/lib/libANN.so tools/_build/libANN_S0.so tiler_amd/lib/libANN.so tools/_build/libANN_S0.so tiler_amd/lib/libANN.so; do
    timeout -k 10 300 python3 -u bench_encoder.py --item-tiles $it --check-kf 1 --lib $L > "$OUT/enc.json" 2> "$OUT/enc.err"
    python3 -c "import json; d=json.loads(open('$OUT/enc.json').read().strip().splitlines()[-1]); print('$L', $it, d['value'], d['wall_s'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['loop_ms_avg'], d['out_digest'], d['parity']['mismatches_total'])" >> "$OUT/ab.txt"
  done
done
echo "ab done"
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_frame_tiling.py tests/test_pipeline.py tests/test_gpu_concurrent.py tests/test_gpu_multidevice.py tests/test_gpu_edges.py tests/test_gpu_orbit.py > "$OUT/tests.log" 2>&1
echo "tests done"

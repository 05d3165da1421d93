#!/usr/bin/env bash
# r06: the device block cache (devmem.hip): the encoder loop's phases, then the GPU tests that create and destroy indexes
set -eu
OUT=gpurun_out/${1:-r06m}
mkdir -p "$OUT"
for it in 16384 0; do
  timeout -k 10 300 python3 -u bench_encoder.py --item-tiles $it --check-kf -1 > "$OUT/enc_$it.json" 2> "$OUT/enc_$it.err"
  python3 -c "import json; d=json.loads(open('$OUT/enc_$it.json').read().strip().splitlines()[-1]); print('items', $it, d['value'], d['wall_s'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['loop_ms_avg'], d['out_digest'])" >> "$OUT/summary.txt"
done
echo "enc done"
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_frame_tiling.py tests/test_gpu_orbit.py tests/test_gpu_multidevice.py tests/test_gpu_concurrent.py \
  tests/test_gpu_scan_small.py tests/test_gpu_list_ties.py tests/test_gpu_kdtree_build.py tests/test_pipeline.py tests/test_gpu_edges.py > "$OUT/tests.log" 2>&1
echo "tests done"

#!/usr/bin/env bash
# r06: orbit detection with a prefix check first (plain PrepareFrameTiling sets skip the full check): encoder loop
# A/B (shot-local and whole-tileset items) against the build before, then the GPU tests that build indexes
set -eu
OUT=gpurun_out/${1:-r06pre}
mkdir -p "$OUT"
for it in 0 16384; do
  for L in tools/_build/libANN_H.so tiler_amd/lib/libANN.so tools/_build/libANN_H.so tiler_amd/lib/libANN.so; do
    timeout -k 10 300 python3 -u bench_encoder.py --item-tiles $it --check-kf -1 --lib $L > "$OUT/enc.json" 2> "$OUT/enc.err"
    python3 -c "import json; d=json.loads(open('$OUT/enc.json').read().strip().splitlines()[-1]); print('$L', $it, d['value'], d['wall_s'], d['prepare_ms_avg'], d['ft_smooth_ms_avg'], d['loop_ms_avg'], d['out_digest'])" >> "$OUT/ab.txt"
  done
done
echo "ab done"
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_orbit.py tests/test_gpu_frame_tiling.py tests/test_pipeline.py tests/test_gpu_kdtree_build.py tests/test_gpu_multidevice.py tests/test_gpu_edges.py > "$OUT/tests.log" 2>&1
echo "tests done"

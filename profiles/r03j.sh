#!/usr/bin/env bash
# Round-3 pass j: generic-path parity tests after the 16-lane rescore, then the 4-keyframe encoder digest (must equal
# r03h's 490242f4597f5801) and its generic rescore time.  Each step has its own limit; set -e.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03j}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_frame_tiling.py tests/test_gpu_edges.py tests/test_gpu_orbit.py tests/test_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests done"
timeout -k 10 200 python3 -u bench_encoder.py --check-kf -1 --frames 96 --no-overlap > "$OUT/enc96.json" 2> "$OUT/enc96.err"
python3 -c "import json; d=json.loads(open('$OUT/enc96.json').read().strip().splitlines()[-1]); print('enc96', d['wall_s'], d['diag']['ft_kernels'].get('nn_rescore'), d['diag']['prepare_kernels'].get('nn_rescore'), d['out_digest'])"
echo "encoder done"

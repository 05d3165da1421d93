#!/usr/bin/env bash
# Round-3 pass b: device PrepareFrameTiling tests, the sustained keyframe-loop line (sequential and overlapped), then
# the experiment-build A/Bs (fused query kernel stores, tier-2 grid).  set -e: the first failure ends it.
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03b
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_frame_tiling.py tests/test_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests done"
timeout -k 10 300 python3 -u bench_encoder.py --no-overlap --check-kf -1 > "$OUT/enc_seq.json" 2> "$OUT/enc_seq.err"
echo "encoder seq done"
timeout -k 10 400 python3 -u bench_encoder.py > "$OUT/enc_ovl.json" 2> "$OUT/enc_ovl.err"
echo "encoder overlap done"
bash profiles/ftq_nt_ab.sh > "$OUT/ab.log" 2>&1
echo "ab done"

set -e
mkdir -p gpurun_out/kf1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_keyframes.py -x -v --timeout 120 --timeout-method thread > gpurun_out/kf1/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 bench.py --steps 2 > gpurun_out/kf1/bench.json 2> gpurun_out/kf1/bench.err
echo bench ok

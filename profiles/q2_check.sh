set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_frame_tiling.py tests/test_gpu_orbit.py tests/test_gpu_edges.py -x -q --timeout 250 --timeout-method thread > gpurun_out/q2_tests.log 2>&1
echo tests ok
cp tiler_amd/lib/libANN.so /tmp/libANN_prod.so
MODES=0 bash profiles/pmode_ab.sh
TILER_FTQ_ONEWAVE=1 MODES=0 bash profiles/pmode_ab.sh
cp /tmp/libANN_prod.so tiler_amd/lib/libANN.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/smprof -o sm -- python3 tools/smooth_probe.py 5 > gpurun_out/smprof.log 2>&1
echo prof ok

set -e
mkdir -p gpurun_out/r04m
cp tiler_amd/lib/libANN.so /tmp/ship.so
for v in experiments var/u8m4 var/u6m8 var/u10m4; do
  cp tiler_amd/lib/$v/libANN.so tiler_amd/lib/libANN.so
  echo "== $v"
  TILER_DL3_PROF=1 timeout -k 10 120 python -u tools/dl3_study.py dump gpurun_out/r04m/$(basename $v).npz 2>&1 | grep -v kmeans_iter
done
cp /tmp/ship.so tiler_amd/lib/libANN.so

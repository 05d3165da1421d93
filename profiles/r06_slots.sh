#!/usr/bin/env bash
# r06: per-tile calls (16 native threads, one handle) with 2 / 3 / 4 coalesced batches in flight per handle
set -eu
OUT=gpurun_out/${1:-r06t}
mkdir -p "$OUT"
for L in tiler_amd/lib/libANN.so tools/_build/libANN_S3.so tools/_build/libANN_S4.so tiler_amd/lib/libANN.so tools/_build/libANN_S3.so tools/_build/libANN_S4.so; do
  timeout -k 10 200 python3 -u tools/percall_probe.py --lib $L --tag $(basename $L) >> "$OUT/percall.txt" 2>> "$OUT/percall.err"
done
echo "percall done"

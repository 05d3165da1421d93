#!/usr/bin/env bash
# r06: per-tile calls, coalescer slots (2 / 3) x follower spin (0 / 200 us): the C5 handle and the C3 / plain handles
set -eu
OUT=gpurun_out/${1:-r06w}
mkdir -p "$OUT"
for L in tiler_amd/lib/libANN.so tools/_build/libANN_S2P200.so tools/_build/libANN_S3P0.so tools/_build/libANN_S2P0.so; do
  timeout -k 10 200 python3 -u tools/c5_percall_ab.py $L $(basename $L) >> "$OUT/c5.txt" 2>> "$OUT/c5.err"
  timeout -k 10 200 python3 -u tools/percall_probe.py --lib $L --tag $(basename $L) >> "$OUT/percall.txt" 2>> "$OUT/percall.err"
done
echo "ab done"

"""Where a farthest-first round's time goes (study tool, not a test).

Runs the C4 K-Modes batch (bench_globaltiling's workload) once with a study build of the library that stamps the 100
MHz real-time counter at 8 points of kmb_ff_persist2 (kmodes.hip, -DTILER_KM_STAMPS), for rounds 64..127 (many bins
alive) and the 64 rounds from Kmax - 128 on (only the largest bin alive), every workgroup:

  0 round start   1 centre known (candidate slots reduced)   2 centre row landed   3 points scanned
  4 best reduced  5 arrival (stores drained, workgroup synced)   6 arrival atomics returned   7 barrier left

    hipcc build:  make -C tiler_amd/csrc EXTRA=-DTILER_KM_STAMPS OUT=$PWD/tools/_build/libANN_kmstamps.so BUILD=/tmp/b
    python3 tools/ff_stamps.py --lib tools/_build/libANN_kmstamps.so

Prints, per window, the median over rounds of the per-phase time (median over workgroups) and of the round length,
and the arrival skew (last arrival - first arrival) and the release latency (first leave - last arrival).
"""
import argparse
import ctypes
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--desired", type=int, default=65536)
    ap.add_argument("--bins", type=int, default=128)
    ap.add_argument("--seed", type=int, default=4)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    import tiler_amd._lib as L
    L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import global_tiling as gt
    from tiler_amd import synth
    from tiler_amd._lib import check
    lib = tiler_amd.load()
    check(lib.tiler_init(0), "tiler_init")
    dev = torch.device("cuda", 0)
    tiles, dith = synth.globaltiling_workload(args.seed, args.n, n_palettes=args.bins)
    lines = gt.write_tile_dataset_line(tiles)
    bins = [np.nonzero(dith == p)[0] for p in range(args.bins)]
    starts, eq = [], []
    for b in bins:
        s = lines[b].astype(np.int64).sum(1)
        starts.append(int(b.size - 1 - np.argmin(s[::-1])) if b.size else 0)
        eq.append(gt.equal_quality_tile_count(b.size))
    share = args.desired / sum(eq)
    run, ks = [], []
    for p, b in enumerate(bins):
        kc = math.ceil(eq[p] * share)
        if b.size > kc:
            run.append(p)
            ks.append(int(round(kc)))
    X = np.ascontiguousarray(np.concatenate([lines[bins[p]] for p in run]))
    off = np.zeros(len(run) + 1, np.int32)
    off[1:] = np.cumsum([bins[p].size for p in run])
    ks = np.array(ks, np.int32)
    st = np.array([starts[p] for p in run], np.int32)
    d_X = torch.from_numpy(X).to(dev)
    d_lab = torch.empty(X.shape[0], dtype=torch.int32, device=dev)
    d_cent = torch.empty((int(ks.sum()), 80), dtype=torch.uint8, device=dev)
    iters = np.zeros(len(run), np.int32)
    costs = np.zeros(len(run), np.uint64)
    vp = ctypes.c_void_p
    p = lambda a: a.ctypes.data_as(vp)  # noqa: E731
    for _ in range(2):  # the second run's stamps are read
        check(lib.tiler_kmodes_batch_dev(vp(d_X.data_ptr()), p(off), len(run), p(ks), p(st), 16, vp(d_lab.data_ptr()),
                                         vp(d_cent.data_ptr()), p(iters), p(costs),
                                         vp(torch.cuda.current_stream(dev).cuda_stream)), "tiler_kmodes_batch_dev")
        torch.cuda.synchronize(dev)
    stamps = np.zeros((2, 64, 256, 8), np.uint64)
    fn = lib.tiler_debug_km_stamps
    fn.argtypes = [vp]
    fn.restype = ctypes.c_int
    assert fn(p(stamps)) == 0
    kmax = int(ks.max())
    out = {"kmax": kmax, "bins": len(run), "largest_bin_rows": int(np.diff(off).max()), "unit": "us (100 MHz counter)",
           "windows": {}}
    names = ["centre known", "row landed", "points scanned", "best reduced", "arrival (drained, synced)",
             "arrival atomics", "barrier left"]
    for w, label in ((0, "rounds 64-127"), (1, f"rounds {kmax - 128}-{kmax - 65} (largest bin only)")):
        s = stamps[w].astype(np.int64)  # [round][wg][pt]
        ok = (s > 0).all(axis=2)
        if not ok.any():
            continue
        rows = {}
        for i in range(1, 8):
            d = (s[:, :, i] - s[:, :, i - 1]) / 100.0  # us
            rows[names[i - 1]] = round(float(np.median(d[ok])), 2)
        rl = (s[1:, :, 0] - s[:-1, :, 0]) / 100.0
        rows["round length"] = round(float(np.median(rl[ok[1:] & ok[:-1]])), 2)
        arr = s[:, :, 5]
        skew = (arr.max(1) - arr.min(1)) / 100.0
        rel = (s[:, :, 7].min(1) - arr.max(1)) / 100.0
        lastleave = (s[:, :, 7].max(1) - s[:, :, 7].min(1)) / 100.0
        rows["arrival skew (last - first arrival)"] = round(float(np.median(skew)), 2)
        rows["release (first leave - last arrival)"] = round(float(np.median(rel)), 2)
        rows["leave skew (last - first leave)"] = round(float(np.median(lastleave)), 2)
        out["windows"][label] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

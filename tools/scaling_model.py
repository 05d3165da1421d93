"""A measured model of the N = 2 / 4 / 8 GPU makespan of the sharded encoder steps (study tool).

The driver's 8-GPU node has not been available, so the scaling curve is unmeasured.  This tool measures, on ONE GPU,
the work each rank would do under the product's own plans (tiler_amd.dist: LPT of the GlobalTiling palette bins by
n x K, of the keyframes by frames x tiles) and reports makespan = the slowest rank's measured time:

* GlobalTiling K-Modes (C4 workload, bench_globaltiling's): for each N and rank, ONE tiler_kmodes_batch_dev call over
  that rank's bins (one untimed run, then timed), so the unsplittable largest bin's floor shows as it would;
* FrameTiling (C3): one keyframe step (bench.py's: 24 frames x 32,400 tiles against 262,144 candidates) timed here,
  times the keyframes per rank of a 1000-frame clip (42 keyframes of 24 frames) under the LPT plan.

It is a model: ranks run one after another on one device, so xGMI traffic, the collectives (merge map MAX, UseCount
SUM, tile streams; a few MB) and per-GPU clock differences are not in it.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kf-ms", type=float, default=0.0, help="measured C3 keyframe step (0: read from --bench)")
    ap.add_argument("--bench", default="", help="a bench.py JSON line to take ms_per_step from")
    args = ap.parse_args()
    import torch
    import tiler_amd
    from tiler_amd import dist as td
    from tiler_amd import global_tiling as gt
    from tiler_amd import synth
    from tiler_amd._lib import check
    lib = tiler_amd.load()
    check(lib.tiler_init(0), "tiler_init")
    dev = torch.device("cuda", 0)
    tiles, dith = synth.globaltiling_workload(4, 1 << 20, n_palettes=128)
    lines = gt.write_tile_dataset_line(tiles)
    bins = [np.nonzero(dith == p)[0] for p in range(128)]
    starts, eq = [], []
    for b in bins:
        s = lines[b].astype(np.int64).sum(1)
        starts.append(int(b.size - 1 - np.argmin(s[::-1])) if b.size else 0)
        eq.append(gt.equal_quality_tile_count(b.size))
    share = 65536 / sum(eq)
    run, ks = [], []
    for p, b in enumerate(bins):
        kc = math.ceil(eq[p] * share)
        if b.size > kc:
            run.append(p)
            ks.append(int(round(kc)))
    sizes = [bins[p].size for p in run]
    vp = ctypes.c_void_p

    def kmodes_time(sel):
        X = np.ascontiguousarray(np.concatenate([lines[bins[run[i]]] for i in sel]))
        off = np.zeros(len(sel) + 1, np.int32)
        off[1:] = np.cumsum([sizes[i] for i in sel])
        k = np.array([ks[i] for i in sel], np.int32)
        st = np.array([starts[run[i]] for i in sel], np.int32)
        d_X = torch.from_numpy(X).to(dev)
        d_lab = torch.empty(X.shape[0], dtype=torch.int32, device=dev)
        d_cent = torch.empty((int(k.sum()), 80), dtype=torch.uint8, device=dev)
        iters = np.zeros(len(sel), np.int32)
        costs = np.zeros(len(sel), np.uint64)
        p = lambda a: a.ctypes.data_as(vp)  # noqa: E731
        out = []
        for _ in range(2):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            check(lib.tiler_kmodes_batch_dev(vp(d_X.data_ptr()), p(off), len(sel), p(k), p(st), 16,
                                             vp(d_lab.data_ptr()), vp(d_cent.data_ptr()), p(iters), p(costs),
                                             vp(torch.cuda.current_stream(dev).cuda_stream)), "tiler_kmodes_batch_dev")
            torch.cuda.synchronize(dev)
            out.append(time.perf_counter() - t0)
        return out[-1]

    li = int(np.argmax(sizes))
    res = {"kmodes": {}, "frametiling": {}}
    t1 = None
    for N in (1, 2, 4, 8):
        plan = td.plan_bins(sizes, ks, N)
        per = [kmodes_time(sel) if sel else 0.0 for sel in plan]
        mk = max(per)
        t1 = mk if N == 1 else t1
        res["kmodes"][str(N)] = {"rank_s": [round(x, 4) for x in per], "makespan_s": round(mk, 4),
                                 "speedup": round(t1 / mk, 3), "bins_per_rank": [len(s) for s in plan],
                                 "largest_bin_rank": int(next(r for r, s in enumerate(plan) if li in s))}
    largest = kmodes_time([li])
    res["kmodes"]["largest_bin_alone_s"] = round(largest, 4)
    res["kmodes"]["largest_bin"] = {"rows": int(sizes[li]), "K": int(ks[li])}
    kf_ms = args.kf_ms
    if not kf_ms and args.bench:
        kf_ms = json.loads(open(args.bench).read().strip().splitlines()[-1])["ms_per_step"]
    if kf_ms:
        kfs = [24] * 41 + [1000 - 41 * 24]
        for N in (1, 2, 4, 8):
            plan = td.plan_keyframes(kfs, 32400, N)
            per = [sum(kfs[u] for u in sel) / 24 * kf_ms for sel in plan]
            res["frametiling"][str(N)] = {"makespan_ms": round(max(per), 2), "keyframes_per_rank": [len(s) for s in plan],
                                          "speedup": round(sum(kfs) / 24 * kf_ms / max(per), 3)}
        res["frametiling"]["keyframe_step_ms"] = kf_ms
    print(json.dumps(res))


if __name__ == "__main__":
    main()

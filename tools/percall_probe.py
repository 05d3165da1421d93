#!/usr/bin/env python3
"""Study script: the reference's per-tile call pattern (ann_kdtree_search once per frame tile from 16 threads on one
handle, main.pas:972 / 4027) through libANN.so's native harness (tiler_debug_percall_bench): calls/s, the median lone
call, batches, and mismatches against the batched search -- on the C3 keyframe handle (262,144 PsyV rows) and on a
12,000-row handle and on the C3 rows shuffled (plain_262144: the same candidates, no mirror orbits, as a real
PrepareFrameTiling set).  --lib selects a library build (A/B)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--queries", type=int, default=8192)
    ap.add_argument("--tag", default="")
    ap.add_argument("--scan-only", action="store_true", help="only the scan-kernel timings on the C3 handle")
    ap.add_argument("--k", type=int, default=1, help="results per call (ann_kdtree_search_multi's cnt for k > 1)")
    args = ap.parse_args()
    import tiler_amd._lib as L
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import synth
    lib = tiler_amd.load()
    L.check(lib.tiler_init(0), "tiler_init")
    rng = np.random.default_rng(12)
    P, T = 128, 65536
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = tiler_amd.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                                flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    wl = synth.make_workload(13, 1920, 1080, 1, 256, n_palettes=8)
    fr = wl.frame_rgb[0].reshape(-1, 64)[:args.queries]
    _, qd = tiler_amd.psyv_batch(rgb=fr, flags=2, want64=False, want32=True)
    qd = np.ascontiguousarray(qd, np.float32)
    vp = ctypes.c_void_p
    out = {"tag": args.tag, "k": args.k}
    for name, data in (() if args.scan_only else
                       (("c3_262144", rows), ("small_12000", rows[rng.choice(rows.shape[0], 12000, replace=False)]),
                        ("plain_262144", rows[rng.permutation(rows.shape[0])]),
                        ("plain_65536", rows[rng.permutation(rows.shape[0])[:65536]]))):
        with tiler_amd.KDTree(data) as kdt:
            bi, be = kdt.search_batch(qd, k=args.k)
            n_idx = np.zeros(qd.shape[0] * args.k, np.int32)
            n_err = np.zeros(qd.shape[0] * args.k, np.float32)
            bi, be = bi.reshape(-1), be.reshape(-1)
            wall, lone = ctypes.c_double(0), ctypes.c_double(0)
            c0 = kdt.combine_stats()
            L.check(lib.tiler_debug_percall_bench(kdt.handle, qd.ctypes.data_as(vp), qd.shape[0], args.k, 16,
                                                  n_idx.ctypes.data_as(vp), n_err.ctypes.data_as(vp),
                                                  ctypes.byref(wall), ctypes.byref(lone)), "percall")
            c1 = kdt.combine_stats()
            nb = c1["batches"] - c0["batches"]
            out[name] = {"calls_per_s": round(qd.shape[0] / wall.value, 1), "lone_us": round(lone.value, 1),
                         "avg_batch": round((c1["calls"] - c0["calls"]) / max(1, nb), 2),
                         "mismatches": int(np.count_nonzero(n_idx != bi) +
                                           np.count_nonzero(n_err.view(np.uint32) != be.view(np.uint32)))}
    # the small-batch scan kernel alone (HIP events): batches of 1, 4 and 16 queries on the C3 handle
    with tiler_amd.KDTree(rows) as kdt:
        for nq in (1, 4, 16):
            kdt.search_batch(qd[:nq])
            lib.tiler_timing_reset()
            lib.tiler_timing_enable(1)
            for r in range(30):
                kdt.search_batch(qd[r * nq:(r + 1) * nq])
            lib.tiler_timing_enable(0)
            n = ctypes.c_int(0)
            ms = lib.tiler_timing_get(b"nn_scan", ctypes.byref(n))
            out[f"scan_us_{nq}q"] = round(1e3 * ms / max(1, n.value), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

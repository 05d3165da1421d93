#!/usr/bin/env python3
"""Debug script: k = 8 on the shuffled C3 rows (a plain 262,144-row handle) -- per-call path (native threads,
coalesced small batches) and batched path, each against the oracle (ANN restated) on the first --queries frame
tiles.  --lib selects a library build."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # the checker (test infrastructure)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--queries", type=int, default=256)
    args = ap.parse_args()
    import tiler_amd._lib as L
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import synth
    import pyoracle
    lib = tiler_amd.load()
    rng = np.random.default_rng(12)
    P, T = 128, 65536
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = tiler_amd.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                                flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    wl = synth.make_workload(13, 1920, 1080, 1, 256, n_palettes=8)
    _, qd = tiler_amd.psyv_batch(rgb=wl.frame_rgb[0].reshape(-1, 64)[:args.queries], flags=2, want64=False,
                                 want32=True)
    qd = np.ascontiguousarray(qd, np.float32)
    rng.choice(rows.shape[0], 12000, replace=False)  # the probe's draw order
    data = np.ascontiguousarray(rows[rng.permutation(rows.shape[0])])
    k, nq = 8, qd.shape[0]
    okd = pyoracle.KDTree(data)
    oi, oe = okd.search_batch(qd, k=k)
    okd.close()
    out = {}
    with tiler_amd.KDTree(data) as kdt:
        bi, be = kdt.search_batch(qd, k=k)
        n_idx = np.zeros(nq * k, np.int32)
        n_err = np.zeros(nq * k, np.float32)
        wall, lone = ctypes.c_double(0), ctypes.c_double(0)
        vp = ctypes.c_void_p
        L.check(lib.tiler_debug_percall_bench(kdt.handle, qd.ctypes.data_as(vp), nq, k, 16, n_idx.ctypes.data_as(vp),
                                              n_err.ctypes.data_as(vp), ctypes.byref(wall), ctypes.byref(lone)),
                "percall")
        small_i, small_e = kdt.search_batch(qd[:16], k=k)  # one small batch through the plain entry point
    for name, gi, ge in (("batched", bi, be), ("percall", n_idx, n_err), ("small16", small_i, small_e)):
        gi = gi.reshape(-1, k)
        ge = ge.reshape(-1, k)
        m = gi.shape[0]
        bad_i = np.nonzero(np.any(gi != oi[:m], axis=1))[0]
        bad_e = np.nonzero(np.any(ge.view(np.uint32) != oe[:m].view(np.uint32), axis=1))[0]
        out[name] = {"queries": int(m), "idx_bad_queries": int(bad_i.size), "err_bad_queries": int(bad_e.size),
                     "first": [int(x) for x in bad_i[:4]]}
        if bad_i.size:
            q0 = int(bad_i[0])
            out[name]["example"] = {"gpu": [int(x) for x in gi[q0]], "oracle": [int(x) for x in oi[q0]],
                                    "gpu_err": [float(x) for x in ge[q0]], "oracle_err": [float(x) for x in oe[q0]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

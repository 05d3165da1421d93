#!/usr/bin/env python3
"""Debug script: one failing k = 8 query of tools/k8_plain_check.py through the small-batch scan alone (nq = 1 and 4)
on the shuffled C3 rows, and the same with the split count reduced (TILER_DEBUG_SCAN_SPLITS), against the oracle."""
import os
import sys

import tiler_amd._lib as L

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # the checker (test infrastructure)


def main():
    import tiler_amd
    from tiler_amd import synth
    import pyoracle
    rng = np.random.default_rng(12)
    P, T = 128, 65536
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = tiler_amd.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                                flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    wl = synth.make_workload(13, 1920, 1080, 1, 256, n_palettes=8)
    _, qd = tiler_amd.psyv_batch(rgb=wl.frame_rgb[0].reshape(-1, 64)[:256], flags=2, want64=False, want32=True)
    qd = np.ascontiguousarray(qd, np.float32)
    rng.choice(rows.shape[0], 12000, replace=False)
    data = np.ascontiguousarray(rows[rng.permutation(rows.shape[0])])
    okd = pyoracle.KDTree(data)
    sel = [4, 6, 17, 22]
    oi, oe = okd.search_batch(qd[sel], k=8)
    okd.close()
    d = ((data - qd[4]) ** 2).sum(1)
    tied = np.nonzero(np.abs(d - oe[0, 0]) < 1e-4)[0]
    print("oracle q4", list(oi[0]), "near-tied rows", list(tied))
    with tiler_amd.KDTree(data) as kdt:
        pos = kdt.positions()
        print("positions of tied", [int(pos[t]) for t in tied])
        for nq in ((1,) if os.environ.get("TILER_DEBUG_DUMP_SCAN") else (1, 4)):
            gi, ge = kdt.search_batch(qd[sel[:nq]], k=8)
            print("nq", nq, "gpu q4", list(gi.reshape(nq, 8)[0]), "ok" if np.array_equal(gi.reshape(nq, 8)[0], oi[0]) else "BAD")
        if os.environ.get("TILER_DEBUG_DUMP_SCAN"):
            raw = np.fromfile(os.environ["TILER_DEBUG_DUMP_SCAN"], np.uint8)
            ns = raw.size // 64
            key = raw[:ns * 32].view(np.float32).reshape(ns, 8)
            idx = raw[ns * 32:].view(np.int32).reshape(ns, 8)
            for t in tied:
                sp = [int(x) for x in np.nonzero(np.any(idx == t, axis=1))[0]]
                print("row", int(t), "in splits", sp, [list(idx[x]) for x in sp][:2])
        lib = tiler_amd.load()
        lib.tiler_set_scan_limits(64, 0)
        gi, ge = kdt.search_batch(qd[sel[:1]], k=8)
        print("mfma path q4", list(gi.reshape(1, 8)[0]))
        lib.tiler_set_scan_limits(64, 16)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Debug script: k = 8 small-batch search on a mirror-orbit index (tests/test_gpu_scan_small.py::
test_scan_small_orbit_index data) against the oracle, printing every query whose lists differ with the sequential fp32
distances of both lists' candidates."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # the checker (test infrastructure)


def seqdist(row, q):
    d = np.float32(0)
    for a, b in zip(q, row):
        t = np.float32(a - b)
        d = np.float32(d + np.float32(t * t))
    return d


def main():
    import tiler_amd
    from tiler_amd import synth
    import pyoracle
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rng = np.random.default_rng(31 + k)
    P, T = 16, 3000
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = tiler_amd.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                                flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    picks = rows[rng.choice(rows.shape[0], 64, replace=False)]
    qs = np.concatenate([picks[:32], picks[32:] + rng.standard_normal((32, 192)).astype(np.float32) * 0.01])
    okd = pyoracle.KDTree(rows, bs=1)
    with tiler_amd.KDTree(rows) as kdt:
        print("groups", kdt.stats()["orbit_groups"], "rows", rows.shape[0])
        for nq in (1, 3):
            q = np.ascontiguousarray(qs[:nq])
            gi, ge = kdt.search_batch(q, k=k)
            oi, oe = okd.search_batch(q, k=k)
            gi, ge, oi, oe = (x.reshape(nq, k) for x in (gi, ge, oi, oe))
            for r in range(nq):
                if np.array_equal(gi[r], oi[r]) and np.array_equal(ge[r].view(np.uint32), oe[r].view(np.uint32)):
                    continue
                print(f"nq {nq} query {r}:")
                print("  gpu   ", list(gi[r]), [float(x) for x in ge[r]])
                print("  oracle", list(oi[r]), [float(x) for x in oe[r]])
                print("  seq(gpu idx)   ", [float(seqdist(rows[j], q[r])) if j >= 0 else None for j in gi[r]])
                print("  seq(oracle idx)", [float(seqdist(rows[j], q[r])) for j in oi[r]])
    okd.close()
    # the first failing pair's neighbourhood alone: 3 groups around rows 6276 / 6278
    for lo in (6272, 6068, 2740):
        sub = np.ascontiguousarray(rows[lo:lo + 12])
        q = np.ascontiguousarray(qs[:3])
        ok2 = pyoracle.KDTree(sub, bs=1)
        with tiler_amd.KDTree(sub) as kdt:
            st = kdt.stats()
            gi, ge = kdt.search_batch(q, k=8)
        oi, oe = ok2.search_batch(q, k=8)
        ok2.close()
        print("subset", lo, "groups", st["orbit_groups"])
        for r in range(3):
            print("  gpu   ", list(gi.reshape(3, 8)[r]), [float(x) for x in ge.reshape(3, 8)[r]])
            print("  oracle", list(oi.reshape(3, 8)[r]), [float(x) for x in oe.reshape(3, 8)[r]])
        print("  rows equal 0-2:", np.array_equal(sub[4], sub[6]), np.array_equal(sub[8], sub[10]),
              np.array_equal(sub[4], sub[5]))


if __name__ == "__main__":
    main()

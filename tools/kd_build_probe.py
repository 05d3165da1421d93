#!/usr/bin/env python3
"""Study script: ann_kdtree_create (create_ms: host wall of the whole index build) and the kd-tree build time (ann_kdtree_create -> kd_build_ms, host wall incl. its device work) on the
encoder's dataset shapes -- the C3 keyframe candidates (262,144 PsyV rows x 192), a shot-local PrepareFrameTiling set
(100,000 x 192), the global 64-d palette-index dataset (262,144 x 64) -- with a digest of the leaf positions.
--lib selects a library build (A/B)."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import tiler_amd._lib as L
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import synth
    lib = tiler_amd.load()
    L.check(lib.tiler_init(0), "tiler_init")
    rng = np.random.default_rng(11)
    P, T = 128, 65536
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = tiler_amd.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                                flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    shapes = {"c3_262144x192": rows, "local_100000x192": rows[rng.choice(rows.shape[0], 100000, replace=False)],
              "global_262144x64": (rng.integers(0, 16, (262144, 64))).astype(np.float32)}
    out = {"tag": args.tag}
    for name, data in shapes.items():
        ms, cms, dig = [], [], None
        for r in range(args.reps + 1):
            t0 = time.perf_counter()
            kdt = tiler_amd.KDTree(data)
            tc = time.perf_counter() - t0
            st = kdt.stats()
            if r:
                ms.append(st["kd_build_ms"])
                cms.append(1e3 * tc)
            if dig is None:
                dig = hashlib.sha256(kdt.positions().tobytes()).hexdigest()[:16]
            kdt.close()
        out[name] = {"best_ms": round(min(ms), 3), "median_ms": round(float(np.median(ms)), 3), "digest": dig,
                     "create_ms": round(float(np.median(cms)), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

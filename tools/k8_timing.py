#!/usr/bin/env python3
"""Timing of PrepareFrameTiling's UseOne preselection (main.pas:3830): k = 8 exact NN of a keyframe's distinct
(palette, tile) items' 64 palette indices in the global 64-d dataset of every tile in 4 orientations
(PrepareGlobalFT main.pas:3763-3779), as the encoder runs it once per keyframe (tiler_prepare_frame_tiling_dev).
C3 shape: 65,536 tiles -> 262,144 rows; --items queries.  Prints the shortlist kernel's HIP-event time (best of
--reps) and a digest of the results.  Study script; not part of the product."""
import argparse
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tag", default="")
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    import torch
    import tiler_amd._lib as L
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import frame_tiling as ftm
    from tiler_amd import synth
    from tiler_amd._lib import check

    lib = tiler_amd.load()
    check(lib.tiler_init(0), "tiler_init")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(20261018)
    tiles, _, _ = synth.tileset(rng, 65536)
    gds = ftm.prepare_global_ft(tiles)
    q = tiles[rng.choice(tiles.shape[0], args.items, replace=False)].astype(np.float32)
    d_q = torch.from_numpy(q).to(dev)
    d_i = torch.empty((args.items, 8), dtype=torch.int32, device=dev)
    d_e = torch.empty((args.items, 8), dtype=torch.float32, device=dev)
    ms = []
    for r in range(args.reps + 1):
        lib.tiler_timing_reset()
        lib.tiler_timing_enable(1 if r else 0)
        gds.kdt.search_batch_dev(d_q.data_ptr(), args.items, 8, d_i.data_ptr(), d_e.data_ptr())
        torch.cuda.synchronize(dev)
        lib.tiler_timing_enable(0)
        if r:
            c = ctypes.c_int(0)
            ms.append(lib.tiler_timing_get(b"nn_shortlist", ctypes.byref(c)))
    h = hashlib.sha256()
    h.update(d_i.cpu().numpy().tobytes())
    h.update(d_e.cpu().numpy().tobytes())
    st = gds.kdt.stats()
    print(json.dumps({"tag": args.tag, "items": args.items, "shortlist_ms": [round(x, 4) for x in ms],
                      "best_ms": round(min(ms), 4), "splits": st["splits"], "fallback": st["fallback_queries"],
                      "exhaustive": st["exhaustive_queries"], "digest": h.hexdigest()[:16]}))
    gds.kdt.close()


if __name__ == "__main__":
    main()

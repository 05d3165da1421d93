#!/usr/bin/env python3
"""Timing modes of the generic 16x16x32 shortlist (nn_shortlist16_kernel) on a real PrepareFrameTiling candidate set.

One keyframe of bench_encoder's clip (1080p, 24 frames, items from --item-tiles tiles of a 64k set, Medium quality):
tiler_prepare_frame_tiling_dev builds its candidate set, then FrameTiling of the keyframe is timed --reps times with
the kernel timers on; prints the shortlist's HIP-event time and the output digest.  With the experiment library and
TILER_SL16_MODE=1..3 the shortlist runs a timing mode (results invalid; the search stops after the shortlist, so
nothing downstream reads them).  Study script (generic shortlist); not part of the product.
"""
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
    ap.add_argument("--item-tiles", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default="")
    ap.add_argument("--lib", default="")
    ap.add_argument("--gate", type=int, default=1, help="the k = 1 insertion gate (tiler_debug_shortlist_gate)")
    args = ap.parse_args()
    import torch
    import tiler_amd._lib as L
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import frame_tiling as ftm
    from tiler_amd import synth
    from tiler_amd._lib import check
    import bench_encoder

    lib = tiler_amd.load()
    check(lib.tiler_init(0), "tiler_init")
    if hasattr(lib, "tiler_debug_shortlist_gate"):
        lib.tiler_debug_shortlist_gate(args.gate)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(20261017)
    P, T, W, H, F = 128, 65536, 1920, 1080, 24
    Q = (W // 8) * (H // 8)
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    tile_pal = rng.integers(0, P, T).astype(np.int32)
    near = ftm.near_palettes(synth.palette_centroids(pals))
    d = {k: torch.from_numpy(np.ascontiguousarray(a)).to(dev) for k, a in
         (("tiles", tiles), ("thm", thm), ("tvm", tvm), ("pals", pals), ("tpal", tile_pal))}
    g = torch.Generator(device=dev)
    g.manual_seed(20261017)
    fr, it = bench_encoder.keyframe_gpu(torch, g, F, Q, T, dev, subset=args.item_tiles)
    ip = d["tpal"][it.long()].int()
    gds = ftm.prepare_global_ft(tiles)
    kt, info = ftm.prepare_frame_tiling_dev(gds, it.data_ptr(), ip.data_ptr(), it.numel(), d["tiles"].data_ptr(),
                                            d["thm"].data_ptr(), d["tvm"].data_ptr(), T, d["pals"].data_ptr(), P, 1,
                                            near, True, -1, 0)
    torch.cuda.synchronize(dev)
    n = F * Q
    out = {nm: torch.empty(n, dtype=dt, device=dev) for nm, dt in
           (("tile", torch.int32), ("pal", torch.int32), ("hm", torch.uint8), ("vm", torch.uint8),
            ("err", torch.float32))}
    vp = ctypes.c_void_p
    ms = []
    for r in range(args.reps + 1):
        lib.tiler_timing_reset()
        lib.tiler_timing_enable(1 if r else 0)
        check(lib.tiler_frame_tiling_dev(kt.handle, vp(fr.data_ptr()), n, 1, -1, vp(out["tile"].data_ptr()),
                                         vp(out["pal"].data_ptr()), vp(out["hm"].data_ptr()), vp(out["vm"].data_ptr()),
                                         vp(out["err"].data_ptr()), vp(0)), "tiler_frame_tiling_dev")
        torch.cuda.synchronize(dev)
        lib.tiler_timing_enable(0)
        if r:
            c = ctypes.c_int(0)
            ms.append(lib.tiler_timing_get(b"nn_shortlist", ctypes.byref(c)))
    st = kt.stats()
    h = hashlib.sha256()
    for nm in ("tile", "pal", "hm", "vm", "err"):
        h.update(out[nm].cpu().numpy().tobytes())
    m0 = info["candidates"]
    flops = 2.0 * (-(-m0 // 16) * 16) * 32 * (6 * (n - st["flat_queries"]) + st["flat_queries"])
    best = min(ms)
    print(json.dumps({"tag": args.tag, "gate": args.gate, "mode": os.environ.get("TILER_SL16_MODE", "0"),
                      "shortlist_ms": ms, "tier2_queries": st["fallback_queries"], "tier3_queries": st["exhaustive_queries"],
                      "candidates": m0, "flat_queries": st["flat_queries"],
                      "frac": round(flops / (best * 1e-3) / 1e12 / 2500.0, 4), "digest": h.hexdigest()[:16]}),
          flush=True)
    kt.close()
    gds.kdt.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Study script: bench.py's C3 FrameTiling step (the headline: 1080p, 24-frame keyframe, 64k tileset x 4 mirrors,
seed 20261015) with a chosen library build (--lib, A/B of kernel variants): step time, the orbit shortlist's HIP-event
time and a digest of the step's tilemap items and errors."""
import argparse
import ctypes
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import torch
    import tiler_amd._lib as L
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    import tiler_amd
    from tiler_amd import synth
    lib = tiler_amd.load()
    L.check(lib.tiler_init(0), "tiler_init")
    dev = torch.device("cuda", 0)
    vp = ctypes.c_void_p
    W, H, F, TS, P = 1920, 1080, 24, 65536, 128
    Q = (W // 8) * (H // 8)
    rng0 = np.random.default_rng(20261015)
    pals = synth.palettes(rng0, P)
    tiles, thm, tvm = synth.tileset(rng0, TS)
    tile_pal = rng0.integers(0, P, TS).astype(np.int32)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
    M = ds.tile_of.size
    frames = synth.keyframe_frames(np.random.default_rng(20261016), F, Q)
    d_rgb = torch.from_numpy(frames.reshape(-1, 64)).to(dev)
    QK = d_rgb.shape[0]
    stream = torch.cuda.current_stream(dev).cuda_stream
    t = {k: torch.from_numpy(v).to(dev) for k, v in (("tiles", tiles), ("pals", pals), ("to", ds.tile_of),
                                                      ("po", ds.pal_of), ("fl", ds.psyv_flags))}
    d_rows = torch.empty((M, 192), dtype=torch.float32, device=dev)
    tiler_amd.psyv_batch_dev(M, palpix=t["tiles"].data_ptr(), tile_of=t["to"].data_ptr(), palettes=t["pals"].data_ptr(),
                             pal_of=t["po"].data_ptr(), flags_per=t["fl"].data_ptr(), flags=1 | 2, gamma=-1,
                             out32=d_rows.data_ptr(), stream=stream)
    torch.cuda.synchronize(dev)
    kdt = tiler_amd.KDTree(dev_ptr=d_rows.data_ptr(), n=M, dd=192, stream=stream)
    L.check(lib.tiler_ft_set_maps(kdt.handle, ds.tile_of.ctypes.data_as(vp), ds.pal_of.ctypes.data_as(vp),
                                  ds.attrs.ctypes.data_as(vp)), "maps")
    out = [torch.empty(QK, dtype=dt, device=dev) for dt in (torch.int32, torch.int32, torch.uint8, torch.uint8,
                                                            torch.float32)]

    def step():
        L.check(lib.tiler_frame_tiling_dev(kdt.handle, vp(d_rgb.data_ptr()), QK, 1, -1,
                                           *[vp(x.data_ptr()) for x in out], vp(stream)), "ft")

    for _ in range(5):
        step()
    torch.cuda.synchronize(dev)
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    lib.tiler_timing_enable(0)
    n = ctypes.c_int(0)
    ms = lib.tiler_timing_get(b"nn_orbit", ctypes.byref(n))
    kern = {}
    for name in ("psyv", "nn_rescore", "nn_pairs", "nn_collect", "kd_verify"):
        c = ctypes.c_int(0)
        t_ = lib.tiler_timing_get(name.encode(), ctypes.byref(c))
        kern[name] = round(t_ / max(1, c.value), 4) if c.value else None
    h = hashlib.sha256()
    for x in out:
        h.update(x.cpu().numpy().tobytes())
    print(json.dumps({"tag": args.tag, "ms_per_step": round(1e3 * el / args.steps, 3),
                      "orbit_ms": round(ms / max(1, n.value), 3), "kernels_ms": kern,
                      "mtiles_s": round(QK * args.steps / el / 1e6, 2),
                      "digest": h.hexdigest()[:16]}), flush=True)
    kdt.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Study of DLv3 pass 2 (palette.hip dl3_reduce_kernel) on bench.py's palette workload (8 frames of a 1080p shot,
128 palettes).  Not part of the product.

  python tools/dl3_study.py dump OUT.npz      (GPU box) DitheringPalIndex of the 8 frames (k-means, GPU) + per-pair
                                               DLv3 table sizes and the phase times
  python tools/dl3_study.py analyze OUT.npz   (host) per-pair sizes, and the restatement's time on the largest pairs
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SEED = 20261015 + 11  # bench.py: args.seed + 11
W, H, F, P = 1920, 1080, 8, 128


def frames():
    from tiler_amd import synth
    pf, _ = synth.shot_frames(np.random.default_rng(SEED), F, W // 8, H // 8, shot_len=(F, F), noise=2)
    return pf


def dump(path):
    import ctypes
    import tiler_amd
    from tiler_amd.palette import prepare_dither_tiles, quantize_palettes
    lib = tiler_amd.load()
    lib.tiler_init(0)
    pf = frames()
    prepare_dither_tiles(pf.reshape(-1, 64), P)  # warm
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    t0 = time.perf_counter()
    lab, _, it = prepare_dither_tiles(pf.reshape(-1, 64), P)
    tk = time.perf_counter() - t0
    lib.tiler_timing_enable(0)
    kp = {}
    for name in ("kmeans", "kmeans_assign", "kmeans_update"):
        n = ctypes.c_int(0)
        kp[name] = round(lib.tiler_timing_get(name.encode(), ctypes.byref(n)), 2)
    print({"prepare_dither_s": round(tk, 3), "kmeans_iterations": it, "kmeans_ms": kp})
    quantize_palettes(pf.reshape(-1, 64), lab, P)  # warm
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    t0 = time.perf_counter()
    pal, uc, colors = quantize_palettes(pf.reshape(-1, 64), lab, P)
    t = time.perf_counter() - t0
    lib.tiler_timing_enable(0)
    ph = {}
    for name in ("dl3_table", "dl3_pass1", "dl3_reduce"):
        n = ctypes.c_int(0)
        ph[name] = lib.tiler_timing_get(name.encode(), ctypes.byref(n))
    np.savez(path, labels=lab, colors=colors, pal=pal, uc=uc)
    print({"s": round(t, 3), "phases_ms": ph, "colors_max": int(colors.max()), "colors_sum": int(colors.sum()),
           "top8": sorted(colors.tolist())[-8:]})


def analyze(path):
    import pyoracle
    z = np.load(path)
    lab, colors = z["labels"], z["colors"]
    pf = frames().reshape(-1, 64)
    order = np.argsort(-colors)
    print("pairs", colors.size, "colors: max", colors.max(), "median", int(np.median(colors)), "sum", colors.sum())
    for p in order[:4]:
        px = pf[lab == p].reshape(-1)
        rgb = np.stack([px & 255, (px >> 8) & 255, (px >> 16) & 255], 1).astype(np.uint8)
        t0 = time.perf_counter()
        out, hist = pyoracle.dl3quant(rgb)
        t = time.perf_counter() - t0
        print(f"pair {p}: pixels {rgb.shape[0]} colors {hist} (gpu {colors[p]}) merges {hist - 16} cpu {t:.2f} s "
              f"palette ok {np.array_equal(np.sort(out), np.sort(z['pal'][p]))}")


if __name__ == "__main__":
    {"dump": dump, "analyze": analyze}[sys.argv[1]](sys.argv[2])

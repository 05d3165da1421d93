#!/usr/bin/env python3
"""Probe: QuantizePalette (DLv3) for many (keyframe, palette) pairs in one call at growing sizes (the stacked-keyframe
form of tiler_quantize_palettes_dev).  Prints per size the time or the library's error.  Study script."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import tiler_amd
    from tiler_amd import synth
    from tiler_amd._lib import check, last_error
    lib = tiler_amd.load()
    check(lib.tiler_init(0), "tiler_init")
    dev = torch.device("cuda", 0)
    vp = ctypes.c_void_p
    for nk in [int(x) for x in sys.argv[1:]] or [2, 4, 8]:
        fr, _ = synth.shot_frames(np.random.default_rng(5), nk * 8, 240, 135, shot_len=(8, 8), noise=2)
        n = fr.shape[0] * fr.shape[1]
        P = 128 * nk
        pal_of = (np.repeat(np.arange(nk), 8 * fr.shape[1]) * 128 +
                  np.random.default_rng(6).integers(0, 128, n)).astype(np.int32)
        d_rgb = torch.from_numpy(fr.reshape(-1, 64)).to(dev)
        d_po = torch.from_numpy(pal_of).to(dev)
        pal = np.zeros((P, 16), np.int32)
        uc = np.zeros(P, np.int32)
        col = np.zeros(P, np.int32)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rc = lib.tiler_quantize_palettes_dev(n, vp(d_rgb.data_ptr()), vp(d_po.data_ptr()), None, P, 16, 7,
                                             pal.ctypes.data_as(vp), uc.ctypes.data_as(vp), col.ctypes.data_as(vp),
                                             None)
        dt = time.perf_counter() - t0
        print(json.dumps({"keyframes": nk, "tiles": n, "pairs": P, "rc": rc, "s": round(dt, 3),
                          "err": last_error() if rc else "", "max_colors": int(col.max())}), flush=True)
        if rc:
            break


if __name__ == "__main__":
    main()

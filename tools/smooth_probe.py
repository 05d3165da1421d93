"""Smooth at C3 shape on the GPU only (for rocprofv3 kernel traces): 24 frames x 32,400 positions of temporally
coherent random items over a 65,536-tile / 128-palette set, tiler_smooth_keyframe_dev called REPS times."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import tiler_amd  # noqa: E402
from tiler_amd import synth  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
F, Q, T, P = 24, 32400, 65536, 128
rng = np.random.default_rng(7)
lib = tiler_amd.load()
dev = torch.device("cuda:0")
palpix = rng.integers(0, 16, (T, 64)).astype(np.uint8)
pals = synth.palettes(rng, P)
tile = np.zeros((F, Q), np.int32)
pal = np.zeros((F, Q), np.int32)
hm = np.zeros((F, Q), np.uint8)
vm = np.zeros((F, Q), np.uint8)
tile[0], pal[0] = rng.integers(0, T, Q), rng.integers(0, P, Q)
for f in range(1, F):
    keep = rng.random(Q) < 0.7
    tile[f] = np.where(keep, tile[f - 1], rng.integers(0, T, Q))
    pal[f] = np.where(keep, pal[f - 1], rng.integers(0, P, Q))
    hm[f] = np.where(keep, hm[f - 1], rng.integers(0, 2, Q))
    vm[f] = np.where(keep, vm[f - 1], rng.integers(0, 2, Q))
d_pp, d_pals = torch.from_numpy(palpix).to(dev), torch.from_numpy(pals).to(dev)
stream = torch.cuda.current_stream(dev).cuda_stream
vp = ctypes.c_void_p
for r in range(REPS):
    t = [torch.from_numpy(x.copy()).to(dev) for x in (tile, pal, hm, vm)]
    sm = torch.zeros((F, Q), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rc = lib.tiler_smooth_keyframe_dev(F, Q, vp(t[0].data_ptr()), None, vp(t[1].data_ptr()), vp(t[2].data_ptr()),
                                       vp(t[3].data_ptr()), vp(sm.data_ptr()), vp(d_pp.data_ptr()),
                                       vp(d_pals.data_ptr()), ctypes.c_double(0.02), vp(stream))
    torch.cuda.synchronize(dev)
    assert rc == 0, tiler_amd._lib.last_error()
    print(f"rep {r}: {(time.perf_counter() - t0) * 1e3:.3f} ms, smoothed {int(sm.sum().item())}", flush=True)

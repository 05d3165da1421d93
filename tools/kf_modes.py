"""Timing experiment: keyframe-correlation kernels (TILER_KF_MODE, see keyframes.hip), 1000 random 1080p frames.
Run once per mode in separate processes (the mode is read once per process)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tiler_amd  # noqa: E402

F, tw, th = int(sys.argv[1]) if len(sys.argv) > 1 else 1000, 240, 135
dev = torch.device("cuda", 0)
clip = torch.randint(0, 1 << 24, (F, tw * th * 64), dtype=torch.int32, device=dev)
lib = tiler_amd.load()
assert lib.tiler_init(0) == 0
corr = np.zeros(F - 1)
s = torch.cuda.current_stream(dev).cuda_stream
best = 1e9
for _ in range(3):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    assert lib.tiler_interframe_correlation_dev(ctypes.c_void_p(clip.data_ptr()), F, tw, th,
                                                corr.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(s)) == 0
    best = min(best, time.perf_counter() - t0)
print(f"mode={os.environ.get('TILER_KF_MODE', '0')} F={F} ms={best * 1e3:.2f} sum={corr.sum():.17g}")

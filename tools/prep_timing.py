"""Timing breakdown of the keyframe Prepare (bench.py prepare(): DoPsyV descriptors + index build + maps) at C3."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tiler_amd  # noqa: E402
from tiler_amd import synth  # noqa: E402

dev = torch.device("cuda", 0)
lib = tiler_amd.load()
assert lib.tiler_init(0) == 0
rng = np.random.default_rng(5)
P, TS = 128, 65536
pals = synth.palettes(rng, P)
tiles, thm, tvm = synth.tileset(rng, TS)
tile_pal = rng.integers(0, P, TS).astype(np.int32)
ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
M = ds.tile_of.size
stream = torch.cuda.current_stream(dev).cuda_stream
d_tiles, d_pals = torch.from_numpy(tiles).to(dev), torch.from_numpy(pals).to(dev)
d_to, d_po, d_fl = (torch.from_numpy(a).to(dev) for a in (ds.tile_of, ds.pal_of, ds.psyv_flags))
vp = ctypes.c_void_p
lib.tiler_timing_enable(1)
for rep in range(3):
    t = [time.perf_counter()]
    d_rows = torch.empty((M, 192), dtype=torch.float32, device=dev)
    tiler_amd.psyv_batch_dev(M, palpix=d_tiles.data_ptr(), tile_of=d_to.data_ptr(), palettes=d_pals.data_ptr(),
                             pal_of=d_po.data_ptr(), flags_per=d_fl.data_ptr(), flags=1 | 2, gamma=-1,
                             out32=d_rows.data_ptr(), stream=stream)
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    kdt = tiler_amd.KDTree(dev_ptr=d_rows.data_ptr(), n=M, dd=192, stream=stream)
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    lib.tiler_ft_set_maps(kdt.handle, ds.tile_of.ctypes.data_as(vp), ds.pal_of.ctypes.data_as(vp),
                          ds.attrs.ctypes.data_as(vp))
    torch.cuda.synchronize(dev)
    t.append(time.perf_counter())
    kdt.close()
    t.append(time.perf_counter())
    print(f"rep {rep}: psyv {1e3*(t[1]-t[0]):.2f} ms, create {1e3*(t[2]-t[1]):.2f} ms, maps {1e3*(t[3]-t[2]):.2f} ms, "
          f"destroy {1e3*(t[4]-t[3]):.2f} ms", flush=True)

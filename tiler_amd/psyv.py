"""PsyV descriptor (ComputeTilePsyVisFeatures, main.pas:2997-3177) through libANN.so."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load

FROM_PAL, WAVELETS, QWEIGHT, HMIRROR, VMIRROR = 1, 2, 8, 16, 32


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def psyv_batch(*, rgb=None, palpix=None, tile_of=None, palettes=None, pal_of=None, flags_per=None, flags: int = 0,
               gamma: int = -1, n: int | None = None, want64: bool = True, want32: bool = False):
    """Descriptors of n tiles on the GPU; returns (out64 [n,192] float64 | None, out32 [n,192] float32 | None)."""
    lib = load()
    rgb = None if rgb is None else np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    palpix = None if palpix is None else np.ascontiguousarray(palpix, np.uint8).reshape(-1, 64)
    tile_of = None if tile_of is None else np.ascontiguousarray(tile_of, np.int32)
    palettes = None if palettes is None else np.ascontiguousarray(palettes, np.int32).reshape(-1, 16)
    pal_of = None if pal_of is None else np.ascontiguousarray(pal_of, np.int32)
    flags_per = None if flags_per is None else np.ascontiguousarray(flags_per, np.uint8)
    if n is None:
        n = rgb.shape[0] if rgb is not None else (tile_of.shape[0] if tile_of is not None else palpix.shape[0])
    out64 = np.zeros((n, 192), np.float64) if want64 else None
    out32 = np.zeros((n, 192), np.float32) if want32 else None
    nt = 0 if palpix is None else palpix.shape[0]
    npal = 0 if palettes is None else palettes.shape[0]
    check(lib.tiler_psyv_batch(n, _p(rgb), nt, _p(palpix), _p(tile_of), npal, _p(palettes), _p(pal_of),
                               _p(flags_per), flags, gamma, _p(out64), _p(out32)), "tiler_psyv_batch")
    return out64, out32


def psyv_batch_dev(n: int, *, rgb=0, palpix=0, tile_of=0, palettes=0, pal_of=0, flags_per=0, flags: int = 0,
                   gamma: int = -1, out64=0, out32=0, stream: int = 0):
    """Device-pointer form (ints are HBM addresses, e.g. torch tensor.data_ptr())."""
    lib = load()
    v = ctypes.c_void_p
    check(lib.tiler_psyv_batch_dev(n, v(rgb or None), v(palpix or None), v(tile_of or None), v(palettes or None),
                                   v(pal_of or None), v(flags_per or None), flags, gamma, v(out64 or None),
                                   v(out32 or None), v(stream or None)), "tiler_psyv_batch_dev")

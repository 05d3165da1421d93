"""Smooth step (btnSmoothClick main.pas:1338-1370 -> DoTemporalSmoothing main.pas:4071-4119) on libANN.so."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load

DEFAULT_STRENGTH = 20 / 1000.0  # seTempoSmoo default 20 (main.lfm:187-196) / 1000 (main.pas:1356)


def smooth_keyframe(tile, pal, hm, vm, smoothed, palpix, palettes, strength: float = DEFAULT_STRENGTH, tmpidx=None):
    """One keyframe's SmoothedTileMap ([F, Q] arrays, initialised from TileMap) smoothed in place on copies;
    returns (tile, pal, hm, vm, smoothed, tmpidx)."""
    lib = load()
    tile = np.array(tile, np.int32, copy=True, order="C")
    pal = np.array(pal, np.int32, copy=True, order="C")
    hm = np.array(hm, np.uint8, copy=True, order="C")
    vm = np.array(vm, np.uint8, copy=True, order="C")
    sm = np.array(smoothed, np.uint8, copy=True, order="C")
    tmp = None if tmpidx is None else np.array(tmpidx, np.int32, copy=True, order="C")
    palpix = np.ascontiguousarray(palpix, np.uint8).reshape(-1, 64)
    palettes = np.ascontiguousarray(palettes, np.int32).reshape(-1, 16)
    F, Q = tile.shape
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    check(lib.tiler_smooth_keyframe(F, Q, p(tile), p(tmp), p(pal), p(hm), p(vm), p(sm), palpix.shape[0], p(palpix),
                                    palettes.shape[0], p(palettes), strength), "tiler_smooth_keyframe")
    return tile, pal, hm, vm, sm, tmp

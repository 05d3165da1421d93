"""Dither step, per tile (FinishDitherTiles main.pas:2482-2544 -> DitherTile main.pas:1998-2055, Thomas Knoll
mixing -- or, with `yliluoma_mix` > 0, the Yliluoma branch main.pas:2055-2067 / 1573-1826 -- + PrepareTileMirrors
main.pas:4049-4069) on libANN.so.  SURVEY.md 8(f)-3.

Palette generation (PrepareDitherTiles' yakmo k-means) and the DitheringPalIndex choice stay outside: the
caller passes the keyframe palettes and each tile's palette index.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def dither_tiles(rgb, pal_of, palettes, yliluoma_mix: int = 0):
    """rgb [n][64] int32 0x00BBGGRR, pal_of [n], palettes [P][palsize] -> (palpix [n][64] u8, hm [n], vm [n]).
    yliluoma_mix = 0: Thomas Knoll mixing (chkUseTK, the reference default); 1..64: Yliluoma mixing with
    FY2MixedColors = yliluoma_mix (cbxYilMix: 1, 2, 4, 8, 16)."""
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    pal_of = np.ascontiguousarray(pal_of, np.int32)
    palettes = np.ascontiguousarray(palettes, np.int32)
    n = rgb.shape[0]
    if pal_of.size != n:
        raise ValueError("dither_tiles: one palette index per tile")
    palpix = np.zeros((n, 64), np.uint8)
    hm = np.zeros(n, np.uint8)
    vm = np.zeros(n, np.uint8)
    if yliluoma_mix:
        check(load().tiler_dither_tiles_yliluoma(n, _p(rgb), _p(pal_of), _p(palettes), palettes.shape[0],
                                                 palettes.shape[1], int(yliluoma_mix), _p(palpix), _p(hm), _p(vm)),
              "tiler_dither_tiles_yliluoma")
    else:
        check(load().tiler_dither_tiles(n, _p(rgb), _p(pal_of), _p(palettes), palettes.shape[0], palettes.shape[1],
                                        _p(palpix), _p(hm), _p(vm)), "tiler_dither_tiles")
    return palpix, hm, vm


def dither_tiles_dev(n: int, d_rgb: int, d_pal_of: int, d_palettes: int, n_palettes: int, palsize: int,
                     d_palpix: int, d_hm: int, d_vm: int, stream=None, yliluoma_mix: int = 0):
    """Same with every array resident in HBM (device pointers), asynchronous on `stream`."""
    v = ctypes.c_void_p
    if yliluoma_mix:
        check(load().tiler_dither_tiles_yliluoma_dev(n, v(d_rgb), v(d_pal_of), v(d_palettes), n_palettes, palsize,
                                                     int(yliluoma_mix), v(d_palpix), v(d_hm), v(d_vm),
                                                     v(stream) if stream else None), "tiler_dither_tiles_yliluoma_dev")
        return
    check(load().tiler_dither_tiles_dev(n, v(d_rgb), v(d_pal_of), v(d_palettes), n_palettes, palsize, v(d_palpix),
                                        v(d_hm), v(d_vm), v(stream) if stream else None), "tiler_dither_tiles_dev")

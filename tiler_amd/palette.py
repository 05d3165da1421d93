"""Palette generation of the Dither step on libANN.so: QuantizePalette with the default Dennis
Lee v3 quantizer for every (keyframe, palette) pair at once (main.pas:2154-2254, 2396-2433; dl3quant,
dlquant/quantizer.c:437-663), and FinishQuantizePalette (main.pas:2435-2480).

Palette pairs are stacked over keyframes (pair = kf * P + palette), as the Dither path stacks keyframe palettes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load

DLV3_BPC = 7  # cbxDLBPC default (main.lfm:502)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def quantize_palettes(rgb, pal_of, n_pairs: int, palsize: int = 16, bpc: int = DLV3_BPC, active=None):
    """rgb [n][64] 0x00BBGGRR tiles, pal_of [n] pair index -> (palettes [n_pairs][palsize] PaletteIndexes in
    CompareCMULHS order, use_count [n_pairs], DLv3 colour-table sizes [n_pairs])."""
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    pal_of = np.ascontiguousarray(pal_of, np.int32)
    if pal_of.size != rgb.shape[0]:
        raise ValueError("quantize_palettes: one pair index per tile")
    act = None if active is None else np.ascontiguousarray(active, np.uint8)
    pal = np.zeros((n_pairs, palsize), np.int32)
    uc = np.zeros(n_pairs, np.int32)
    colors = np.zeros(n_pairs, np.int32)
    check(load().tiler_quantize_palettes(rgb.shape[0], _p(rgb), _p(pal_of), _p(act), n_pairs, palsize, bpc, _p(pal),
                                         _p(uc), _p(colors)), "tiler_quantize_palettes")
    return pal, uc, colors


def finish_quantize_order(use_count) -> np.ndarray:
    """lut[old palette] = new palette (FinishQuantizePalette's sort by use count, main.pas:2444-2455)."""
    uc = np.ascontiguousarray(use_count, np.int32)
    lut = np.zeros(uc.size, np.int32)
    check(load().tiler_finish_quantize_order(uc.size, _p(uc), _p(lut)), "tiler_finish_quantize_order")
    return lut


def finish_quantize_palette(palettes, use_count, dith_pal, centroids=None):
    """FinishQuantizePalette for one keyframe: palettes [P][16] reordered by use count, every tile's
    DitheringPalIndex remapped, the palette centroids permuted alike (main.pas:2444-2479)."""
    lut = finish_quantize_order(use_count)
    palettes = np.asarray(palettes)
    new_pal = np.empty_like(palettes)
    new_pal[lut] = palettes
    new_dith = lut[np.asarray(dith_pal, np.int64)]
    new_cent = None
    if centroids is not None:
        centroids = np.asarray(centroids)
        new_cent = np.empty_like(centroids)
        new_cent[lut] = centroids
    return new_pal, new_dith, new_cent, lut

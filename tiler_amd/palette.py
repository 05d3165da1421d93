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


def kmeans(X, k: int, max_iter: int = 0, seed: int = 0):
    """The Dither step's k-means over X [n][d] fp64 (d <= 192) -> (labels [n], centroids [k][d], assignments)."""
    X = np.ascontiguousarray(X, np.float64)
    n, d = X.shape
    labels = np.zeros(n, np.int32)
    cent = np.zeros((k, d), np.float64)
    it = ctypes.c_int(0)
    check(load().tiler_kmeans(_p(X), n, d, k, max_iter, seed, _p(labels), _p(cent), ctypes.byref(it)), "tiler_kmeans")
    return labels, cent, it.value


def prepare_dither_tiles(rgb, n_palettes: int, gamma: int = -1, use_wavelets: bool = True, max_iter: int = 0,
                         seed: int = 0):
    """PrepareDitherTiles for one keyframe (main.pas:2097-2152): its tiles rgb [n][64] (frame order) ->
    (DitheringPalIndex [n], PaletteCentroids [n_palettes][192], Lloyd assignments)."""
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    labels = np.zeros(rgb.shape[0], np.int32)
    cent = np.zeros((n_palettes, 192), np.float64)
    it = ctypes.c_int(0)
    check(load().tiler_prepare_dither_tiles(rgb.shape[0], _p(rgb), n_palettes, gamma, 1 if use_wavelets else 0,
                                            max_iter, seed, _p(labels), _p(cent), ctypes.byref(it)),
          "tiler_prepare_dither_tiles")
    return labels, cent, it.value


def generate_palettes(frames, kf_start, n_palettes: int, palsize: int = 16, gamma: int = -1,
                      use_wavelets: bool = True, bpc: int = DLV3_BPC, max_iter: int = 0):
    """The palette half of btnDitherClick (main.pas:886-907) over all keyframes: PrepareDitherTiles per keyframe,
    QuantizePalette for every (keyframe, palette) pair in one GPU pass, FinishQuantizePalette per keyframe.
    frames [F][Q][64] RGB, kf_start [KF+1] -> (palettes [KF][P][palsize], centroids [KF][P][192],
    DitheringPalIndex [F*Q], use counts [KF][P])."""
    frames = np.ascontiguousarray(frames, np.int32)
    F, Q = frames.shape[:2]
    kf_start = np.asarray(kf_start, np.int64)
    KF, P = kf_start.size - 1, n_palettes
    dith = np.zeros(F * Q, np.int32)
    cent = np.zeros((KF, P, 192), np.float64)
    for k in range(KF):
        f0, f1 = int(kf_start[k]), int(kf_start[k + 1])
        lab, c, _ = prepare_dither_tiles(frames[f0:f1].reshape(-1, 64), P, gamma, use_wavelets, max_iter)
        dith[f0 * Q:f1 * Q] = lab
        cent[k] = c
    kf_of_tile = np.repeat(np.repeat(np.arange(KF), np.diff(kf_start)), Q)
    pal, uc, _ = quantize_palettes(frames.reshape(-1, 64), (kf_of_tile * P + dith).astype(np.int32), KF * P, palsize,
                                   bpc)
    pal = pal.reshape(KF, P, palsize)
    uc = uc.reshape(KF, P)
    for k in range(KF):
        f0, f1 = int(kf_start[k]), int(kf_start[k + 1])
        pal[k], dith[f0 * Q:f1 * Q], cent[k], lut = finish_quantize_palette(pal[k], uc[k], dith[f0 * Q:f1 * Q],
                                                                             cent[k])
        u2 = np.empty_like(uc[k])
        u2[lut] = uc[k]
        uc[k] = u2
    return pal, cent, dith, uc

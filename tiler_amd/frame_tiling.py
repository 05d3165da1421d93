"""FrameTiling step (btnDoFrameTilingClick main.pas:945-977) on libANN.so.

Mirrors the reference's procedures with the same names and argument meaning:
  prepare_global_ft      PrepareGlobalFT      main.pas:3736-3780   (64-d palette-index rows, 4 orientations)
  prepare_frame_tiling   PrepareFrameTiling   main.pas:3791-3967   (k=8 preselection -> used -> DoPsyV dataset)
  do_frame_tiling        DoFrameTiling        main.pas:3992-4047   (query descriptor -> exact NN -> tilemap)
  finish_frame_tiling    FinishFrameTiling    main.pas:3969-3990
The searches and descriptors run on the GPU; the host keeps only the used-table bookkeeping.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import check, load
from .ann import KDTree
from .psyv import FROM_PAL, WAVELETS, psyv_batch
from .synth import FTDataset, ft_dataset_from_used, hflip, vflip

FT_FAST, FT_MEDIUM, FT_SLOW = 0, 1, 2
CFT_PALETTE_TOL = 0.05  # cFTPaletteTol main.pas:23


@dataclass
class GlobalDS:
    kdt: KDTree
    tr_tile: np.ndarray
    tr_attrs: np.ndarray


def prepare_global_ft(tiles: np.ndarray, active: np.ndarray | None = None) -> GlobalDS:
    """PrepareGlobalFT: per active tile rows (F), (H), (H+V), (V) with attrs 0, 1, 3, 2 (main.pas:3763-3777)."""
    tiles = np.asarray(tiles, np.uint8).reshape(-1, 64)
    idx = np.arange(tiles.shape[0]) if active is None else np.nonzero(active)[0]
    t0 = tiles[idx]
    t1 = hflip(t0)
    t2 = vflip(t1)
    t3 = hflip(t2)
    rows = np.stack([t0, t1, t2, t3], 1).reshape(-1, 64).astype(np.float32)
    tr_tile = np.repeat(idx.astype(np.int32), 4)
    tr_attrs = np.tile(np.array([0, 1, 3, 2], np.uint8), idx.size)
    kdt = KDTree(rows)
    if tr_tile.size:  # TRToTileIdx / TRToAttrs on the device too (tiler_prepare_frame_tiling_dev reads them)
        v = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        check(load().tiler_ft_set_maps(kdt.handle, v(tr_tile), v(np.zeros_like(tr_tile)), v(tr_attrs)),
              "tiler_ft_set_maps")
    return GlobalDS(kdt, tr_tile, tr_attrs)


def palette_corr(centroids: np.ndarray):
    """BuildPaletteCorrTriangle main.pas:3855-3867 (CompareEuclideanDCTPtr: sequential double sums)."""
    c = np.asarray(centroids, np.float64)
    P = c.shape[0]
    corr = np.zeros((P, P))
    for k in range(c.shape[1]):  # dimension order, like the reference's pointer walk
        d = c[:, None, k] - c[None, :, k]
        corr += d * d
    finite = corr[~np.isnan(corr)]
    highest = max(0.0, float(finite.max())) if finite.size else 0.0
    return corr, highest


def mark_used(gds: GlobalDS, tiles: np.ndarray, item_pal: np.ndarray, item_tile: np.ndarray, n_palettes: int,
              quality: int = FT_MEDIUM, corrs=None, highest: float = 0.0, paltol: float = CFT_PALETTE_TOL):
    """PrepareFrameTiling.UseOne over every tilemap item of the keyframe (main.pas:3802-3853):
    k=8 exact NN of the tile's 64 indices; walk ascending, skip results whose err equals the previous."""
    tiles = np.asarray(tiles, np.uint8).reshape(-1, 64)
    T = tiles.shape[0]
    used = np.zeros((n_palettes, T, 4), np.uint8)
    keys = np.unique(np.asarray(item_pal, np.int64) * T + np.asarray(item_tile, np.int64))
    if keys.size == 0:
        return used
    pal = (keys // T).astype(np.int64)
    til = (keys % T).astype(np.int64)
    idxs, errs = gds.kdt.search_batch(tiles[til].astype(np.float32), k=8)
    prev = np.full(keys.size, np.inf, np.float64)
    for j in range(8):
        e = errs[:, j].astype(np.float64)
        take = (e != prev) & (idxs[:, j] >= 0)
        prev = e
        r = idxs[take, j]
        t_i, a_i, p_i = gds.tr_tile[r], gds.tr_attrs[r], pal[take]
        if quality == FT_FAST:
            used[p_i, t_i, a_i] = 1
        elif quality == FT_MEDIUM:
            ok = corrs[:, p_i] < paltol * highest  # [P, sel]
            pp, ss = np.nonzero(ok)
            used[pp, t_i[ss], a_i[ss]] = 1
        else:
            used[:, t_i, a_i] = 1
    return used


class KeyframeTiler:
    """The keyframe's TTilingDataset (main.pas:181-189) held in HBM: candidate descriptors (DoPsyV),
    the search index and the TRTo* maps.  `do_frame_tiling` is DoFrameTiling for a batch of frames."""

    def __init__(self, tiles, thm, tvm, palettes, ds: FTDataset, use_wavelets: bool = True, gamma: int = -1):
        self.use_wavelets = use_wavelets
        self.gamma = gamma
        self.ds = ds
        flags = FROM_PAL | (WAVELETS if use_wavelets else 0)
        _, rows = psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=palettes, pal_of=ds.pal_of,
                             flags_per=ds.psyv_flags, flags=flags, gamma=gamma, want64=False, want32=True)
        self.rows = rows
        self.kdt = KDTree(rows)
        lib = load()
        check(lib.tiler_ft_set_maps(self.kdt.handle, ds.tile_of.ctypes.data_as(ctypes.c_void_p),
                                    ds.pal_of.ctypes.data_as(ctypes.c_void_p),
                                    ds.attrs.ctypes.data_as(ctypes.c_void_p)), "tiler_ft_set_maps")

    @property
    def knn_size(self) -> int:
        return int(self.ds.tile_of.size)

    def do_frame_tiling(self, frame_rgb: np.ndarray):
        """frame_rgb [Q, 64] (or [F, Q, 64]) -> (tile, pal, hmirror, vmirror, err)."""
        lib = load()
        rgb = np.ascontiguousarray(frame_rgb, np.int32).reshape(-1, 64)
        Q = rgb.shape[0]
        tile = np.zeros(Q, np.int32)
        pal = np.zeros(Q, np.int32)
        hm = np.zeros(Q, np.uint8)
        vm = np.zeros(Q, np.uint8)
        err = np.zeros(Q, np.float32)
        v = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        check(lib.tiler_frame_tiling(self.kdt.handle, v(rgb), Q, int(self.use_wavelets), self.gamma, v(tile), v(pal),
                                     v(hm), v(vm), v(err)), "tiler_frame_tiling")
        return tile, pal, hm, vm, err

    def finish_frame_tiling(self):
        self.kdt.close()


def prepare_frame_tiling(tiles, thm, tvm, palettes, gds: GlobalDS, item_pal, item_tile, quality: int = FT_MEDIUM,
                         palette_centroids=None, use_wavelets: bool = True, gamma: int = -1) -> KeyframeTiler:
    """PrepareFrameTiling main.pas:3791-3967: used table -> DoPsyV dataset -> index."""
    P = np.asarray(palettes).reshape(-1, 16).shape[0]
    corrs, highest = (None, 0.0)
    if quality == FT_MEDIUM:
        corrs, highest = palette_corr(palette_centroids)
    used = mark_used(gds, tiles, item_pal, item_tile, P, quality, corrs, highest)
    ds = ft_dataset_from_used(used, np.asarray(thm, np.uint8), np.asarray(tvm, np.uint8))
    return KeyframeTiler(tiles, thm, tvm, palettes, ds, use_wavelets, gamma)


def near_palettes(palette_centroids, paltol: float = CFT_PALETTE_TOL) -> np.ndarray:
    """Medium quality's palette pairs (UseOne main.pas:3838-3846): near[p', p] = corr(p', p) < tol * HighestCorr."""
    corrs, highest = palette_corr(palette_centroids)
    return np.ascontiguousarray((corrs < paltol * highest).astype(np.uint8))


def prepare_frame_tiling_dev(gds: GlobalDS, d_item_tile: int, d_item_pal: int, n_items: int, d_palpix: int,
                             d_thm: int, d_tvm: int, n_tiles: int, d_palettes: int, n_palettes: int,
                             quality: int = FT_MEDIUM, near: np.ndarray | None = None, use_wavelets: bool = True,
                             gamma: int = -1, stream: int = 0):
    """PrepareFrameTiling main.pas:3791-3967 on the device (tiler_prepare_frame_tiling_dev): the keyframe's
    tilemap items (HBM int32 pointers) -> UseOne's k = 8 preselection -> used -> DoPsyV dataset -> search handle.
    Returns (KDTree over the keyframe's candidates with its maps set, {"items", "candidates"})."""
    from ._lib import PrepareInfo
    lib = load()
    info = PrepareInfo()
    nr = None
    if quality == FT_MEDIUM:
        if near is None:
            raise ValueError("Medium quality needs the near-palette table (near_palettes)")
        nr = np.ascontiguousarray(near, np.uint8)
    vp = ctypes.c_void_p
    h = lib.tiler_prepare_frame_tiling_dev(gds.kdt.handle, vp(d_item_tile), vp(d_item_pal), int(n_items),
                                           vp(d_palpix), vp(d_thm), vp(d_tvm), int(n_tiles), vp(d_palettes),
                                           int(n_palettes), int(quality),
                                           nr.ctypes.data_as(vp) if nr is not None else None, int(use_wavelets),
                                           int(gamma), vp(stream), ctypes.byref(info))
    if not h:
        check(-1, "tiler_prepare_frame_tiling_dev")
    return KDTree.adopt(h, info.candidates, 192), {"items": int(info.items), "candidates": int(info.candidates)}

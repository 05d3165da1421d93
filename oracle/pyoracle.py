"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so (the CPU restatement).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker.  The product (tiler_amd / libANN.so) never imports it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libkmodes_ref.so")

_o = None


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _threads() -> int:
    """Worker threads of the CPU restatement: the visible cores, capped at 16 (a GPU box's CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def lib():
    global _o
    if _o is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle` (or __graft_entry__.build())")
        _o = ctypes.CDLL(LIB)
        _o.or_km_dissim.restype = ctypes.c_uint64
        _o.or_km_dissim_generic.restype = ctypes.c_uint64
        _o.or_randint.restype = ctypes.c_uint32
        _o.or_palette_corr.restype = ctypes.c_double
        _o.or_dist.restype = ctypes.c_float
        _o.or_dct_lut.restype = ctypes.c_void_p
        _o.or_gamma_lut.restype = ctypes.c_void_p
        _o.or_set_gamma.argtypes = [ctypes.c_double, ctypes.c_double]
        _o.or_smooth.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 8 + [ctypes.c_double]
        _o.or_eqtc.argtypes = [ctypes.c_double]
        _o.or_interframe_corr.restype = ctypes.c_double
        _o.or_init()
    return _o


def psyv(rgb=None, palpix=None, pal=None, flags=0, gamma=-1):
    out = np.zeros(192, np.float64)
    rgb = None if rgb is None else np.ascontiguousarray(rgb, np.int32)
    palpix = None if palpix is None else np.ascontiguousarray(palpix, np.uint8)
    pal = None if pal is None else np.ascontiguousarray(pal, np.int32)
    lib().or_psyv(_p(rgb), _p(palpix), _p(pal), flags, gamma, _p(out))
    return out


def psyv_batch(n, rgb=None, palpix=None, pals=None, pal_of=None, flags_per=None, flags=0, gamma=-1):
    """pal mode: palpix is [n,64] (already gathered per item)."""
    out = np.zeros((n, 192), np.float64)
    a = [None if x is None else np.ascontiguousarray(x) for x in (rgb, palpix, pals, pal_of, flags_per)]
    if a[0] is not None:
        a[0] = a[0].astype(np.int32)
    if a[1] is not None:
        a[1] = a[1].astype(np.uint8)
    if a[2] is not None:
        a[2] = a[2].astype(np.int32)
    if a[3] is not None:
        a[3] = a[3].astype(np.int32)
    if a[4] is not None:
        a[4] = a[4].astype(np.uint8)
    lib().or_psyv_batch(n, *[_p(x) for x in a], flags, gamma, _p(out))
    return out


def nn(data, q):
    data = np.ascontiguousarray(data, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    err = np.zeros(1, np.float32)
    i = lib().or_nn(_p(data), data.shape[0], data.shape[1], _p(q), _p(err))
    return i, float(err[0])


def knn(data, q, k):
    data = np.ascontiguousarray(data, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    idx = np.zeros(k, np.int32)
    err = np.zeros(k, np.float32)
    lib().or_knn(_p(data), data.shape[0], data.shape[1], _p(q), k, _p(idx), _p(err))
    return idx, err


def nn_batch(data, qs, threads=None):
    data = np.ascontiguousarray(data, np.float32)
    qs = np.ascontiguousarray(qs, np.float32).reshape(-1, data.shape[1])
    idx = np.zeros(qs.shape[0], np.int32)
    err = np.zeros(qs.shape[0], np.float32)
    lib().or_nn_batch(_p(data), data.shape[0], data.shape[1], _p(qs), qs.shape[0], _p(idx), _p(err),
                      threads or _threads())
    return idx, err


class KDTree:
    """The reference's CPU search: ANN 1.1.2 kd-tree (ann_kdtree.c; ANN_KD_STD, bucket bs, eps = 0)."""

    def __init__(self, data, bs: int = 1):
        self.data = np.ascontiguousarray(data, np.float32)
        f = lib().or_kdtree_build_bs
        f.restype = ctypes.c_void_p
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        self.h = f(_p(self.data), self.data.shape[0], self.data.shape[1], bs)
        self.visited = 0

    def search_batch(self, qs, threads=None, k: int = 1):
        """annkSearch per query: k = 1 -> (idx[nq], err[nq]); k > 1 -> ([nq, k], [nq, k]) ascending."""
        qs = np.ascontiguousarray(qs, np.float32).reshape(-1, self.data.shape[1])
        idx = np.zeros((qs.shape[0], k), np.int32)
        err = np.zeros((qs.shape[0], k), np.float32)
        f = lib().or_kdtree_search_multi_batch
        f.restype = ctypes.c_long
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_int]
        self.visited += f(self.h, _p(qs), qs.shape[0], k, _p(idx), _p(err), threads or _threads())
        return (idx[:, 0], err[:, 0]) if k == 1 else (idx, err)

    def pri_search_batch(self, qs, eps: float = 0.0):
        """annkPriSearch per query (k = 1, ann_kdtree_pri_search): (idx[nq], err[nq])"""
        qs = np.ascontiguousarray(qs, np.float32).reshape(-1, self.data.shape[1])
        idx = np.zeros(qs.shape[0], np.int32)
        err = np.zeros(qs.shape[0], np.float32)
        f = lib().or_kdtree_pri_search_batch
        f.restype = None
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
                      ctypes.c_void_p]
        f(self.h, _p(qs), qs.shape[0], eps, _p(idx), _p(err))
        return idx, err

    def splits(self):
        """split nodes by split position m: (cut_dim, cut_val, lo_bnd, hi_bnd), arrays [n] (index 0 unused)"""
        n = self.data.shape[0]
        cd = np.zeros(n, np.int32)
        cv, lo, hi = (np.zeros(n, np.float32) for _ in range(3))
        f = lib().or_kdtree_splits
        f.argtypes = [ctypes.c_void_p] * 5
        f(self.h, _p(cd), _p(cv), _p(lo), _p(hi))
        return cd, cv, lo, hi

    def positions(self):
        """leaf position of every point (pos[pidx[i]] = i)"""
        pos = np.zeros(self.data.shape[0], np.int32)
        f = lib().or_kdtree_positions
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        f(self.h, _p(pos))
        return pos

    def close(self):
        if self.h:
            f = lib().or_kdtree_free
            f.argtypes = [ctypes.c_void_p]
            f(self.h)
            self.h = None

    def __del__(self):
        self.close()


def build_ft_dataset(used, palpix, thm, tvm, palettes, use_wavelets=True, gamma=-1):
    used = np.ascontiguousarray(used, np.uint8)
    P, T, _ = used.shape
    cnt = int(used.sum())
    ds = np.zeros((max(cnt, 1), 192), np.float32)
    tidx = np.zeros(max(cnt, 1), np.int32)
    pidx = np.zeros(max(cnt, 1), np.int32)
    attrs = np.zeros(max(cnt, 1), np.uint8)
    n = lib().or_build_ft_dataset(_p(used), P, T, _p(np.ascontiguousarray(palpix, np.uint8)),
                                  _p(np.ascontiguousarray(thm, np.uint8)), _p(np.ascontiguousarray(tvm, np.uint8)),
                                  _p(np.ascontiguousarray(palettes, np.int32)), int(use_wavelets), gamma, _p(ds),
                                  _p(tidx), _p(pidx), _p(attrs))
    return ds[:n], tidx[:n], pidx[:n], attrs[:n]


def frame_tiling(frame_rgb, ds, tidx, pidx, attrs, use_wavelets=True, gamma=-1, threads=None, kd_order=True):
    """DoFrameTiling; kd_order: ties as ANN's kd-tree search returns them (the reference), else lowest index."""
    rgb = np.ascontiguousarray(frame_rgb, np.int32).reshape(-1, 64)
    Q = rgb.shape[0]
    out = [np.zeros(Q, np.int32), np.zeros(Q, np.int32), np.zeros(Q, np.uint8), np.zeros(Q, np.uint8),
           np.zeros(Q, np.float32)]
    lib().or_frame_tiling(_p(rgb), Q, _p(np.ascontiguousarray(ds, np.float32)), ds.shape[0], _p(tidx), _p(pidx),
                          _p(attrs), int(use_wavelets), gamma, threads or _threads(), int(bool(kd_order)),
                          *[_p(o) for o in out])
    return tuple(out)


def prepare_global_ds(palpix, active=None):
    palpix = np.ascontiguousarray(palpix, np.uint8)
    T = palpix.shape[0]
    active = np.ones(T, np.uint8) if active is None else np.ascontiguousarray(active, np.uint8)
    ds = np.zeros((4 * T, 64), np.float32)
    ti = np.zeros(4 * T, np.int32)
    at = np.zeros(4 * T, np.uint8)
    n = lib().or_prepare_global_ds(_p(palpix), _p(active), T, _p(ds), _p(ti), _p(at))
    return ds[:n], ti[:n], at[:n]


def palette_corr(centroids):
    c = np.ascontiguousarray(centroids, np.float64)
    P = c.shape[0]
    corr = np.zeros((P, P), np.float64)
    hi = lib().or_palette_corr(_p(c), P, _p(corr))
    return corr, hi


def mark_used(gds, g_tile, g_attr, item_pal, item_tile, palpix, P, quality, corrs=None, highest=0.0, paltol=0.05,
              kd_order=True):
    palpix = np.ascontiguousarray(palpix, np.uint8)
    T = palpix.shape[0]
    used = np.zeros((P, T, 4), np.uint8)
    corrs = np.zeros((P, P)) if corrs is None else np.ascontiguousarray(corrs, np.float64)
    item_pal = np.ascontiguousarray(item_pal, np.int32)
    item_tile = np.ascontiguousarray(item_tile, np.int32)
    f = lib().or_mark_used
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                  ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
    f(_p(np.ascontiguousarray(gds, np.float32)), gds.shape[0], _p(np.ascontiguousarray(g_tile, np.int32)),
      _p(np.ascontiguousarray(g_attr, np.uint8)), _p(item_pal), _p(item_tile), item_pal.size, _p(palpix), T, P,
      quality, _p(corrs), highest, paltol, int(bool(kd_order)), _p(used))
    return used


def smooth(tile, pal, hm, vm, smoothed, palpix, palettes, strength=0.02, tmpidx=None):
    """In place on copies; arrays [F, Q]."""
    tile = np.array(tile, np.int32, copy=True)
    pal = np.array(pal, np.int32, copy=True)
    hm = np.array(hm, np.uint8, copy=True)
    vm = np.array(vm, np.uint8, copy=True)
    smoothed = np.array(smoothed, np.uint8, copy=True)
    tmp = None if tmpidx is None else np.array(tmpidx, np.int32, copy=True)
    F, Q = tile.shape
    lib().or_smooth(F, Q, _p(tile), _p(tmp), _p(pal), _p(hm), _p(vm), _p(smoothed),
                    _p(np.ascontiguousarray(palpix, np.uint8)), _p(np.ascontiguousarray(palettes, np.int32)),
                    strength)
    return tile, pal, hm, vm, smoothed, tmp


def km_dissim(row, item):
    return int(lib().or_km_dissim(_p(np.ascontiguousarray(row, np.uint8)), _p(np.ascontiguousarray(item, np.uint8))))


def km_get_min(rows, item):
    rows = np.ascontiguousarray(rows, np.uint8)
    best = ctypes.c_uint64()
    i = lib().or_km_get_min(_p(rows), rows.shape[0], _p(np.ascontiguousarray(item, np.uint8)), ctypes.byref(best))
    return i, best.value


def kmodes(X, k, start, modalities=16, threads=1):
    """ComputeKModes; threads > 1 splits the distance loops (results do not depend on it)."""
    lib().or_set_threads(int(threads))
    X = np.ascontiguousarray(X, np.uint8)
    n, a = X.shape
    labels = np.zeros(n, np.int32)
    cent = np.zeros((k, a), np.uint8)
    it = ctypes.c_int()
    cost = ctypes.c_uint64()
    lib().or_kmodes(_p(X), n, a, k, start, modalities, _p(labels), _p(cent), ctypes.byref(it), ctypes.byref(cost))
    return labels, cent, it.value, cost.value


def randint(rng_range, seed):
    s = ctypes.c_uint32(seed)
    r = lib().or_randint(ctypes.c_uint32(rng_range), ctypes.byref(s))
    return r, s.value


def make_tiles_unique(palpix, active, use_count):
    """or_make_tiles_unique on copies: (palpix, active, use_count, merge_index)."""
    palpix = np.array(palpix, np.uint8, copy=True, order="C")
    active = np.array(active, np.uint8, copy=True)
    uc = np.array(use_count, np.int32, copy=True)
    mi = np.full(palpix.shape[0], -1, np.int32)
    lib().or_make_tiles_unique(palpix.shape[0], _p(palpix), _p(active), _p(uc), _p(mi))
    return palpix, active, uc, mi


def reindex(active, use_count):
    active = np.ascontiguousarray(active, np.uint8)
    idx = np.zeros(active.shape[0], np.int32)
    lib().or_reindex(active.shape[0], _p(active), _p(np.ascontiguousarray(use_count, np.int32)), _p(idx))
    return idx


def global_tiling(palpix, dith_pal, P, desired, palsize=16, restart=7, use_count=None, active=None):
    palpix = np.array(palpix, np.uint8, copy=True)
    T = palpix.shape[0]
    active = np.ones(T, np.uint8) if active is None else np.array(active, np.uint8, copy=True)
    uc = np.ones(T, np.int32) if use_count is None else np.array(use_count, np.int32, copy=True)
    mi = np.full(T, -1, np.int32)
    kpb = np.zeros(P, np.int32)
    lib().or_global_tiling(T, _p(palpix), _p(active), _p(uc), _p(mi), _p(np.ascontiguousarray(dith_pal, np.int32)), P,
                           palsize, desired, restart, _p(kpb))
    return palpix, active, uc, mi, kpb


def interframe_corr_batch(frames, tm_w, tm_h):
    """ComputeInterFrameCorrelation (main.pas:811-828) of every consecutive pair: corr[i-1] = corr(i-1, i)."""
    frames = np.ascontiguousarray(frames, np.int32).reshape(-1, tm_w * tm_h * 64)
    F = frames.shape[0]
    corr = np.zeros(max(0, F - 1), np.float64)
    if F > 1:
        lib().or_interframe_corr_batch(_p(frames), F, tm_w, tm_h, _p(corr))
    return corr


def find_keyframes(corr, F, tile_map_size):
    """btnLoadClick main.pas:1099-1146: keyframe index per frame and the keyframe count."""
    corr = np.ascontiguousarray(corr, np.float64)
    kf = np.zeros(F, np.int32)
    n = lib().or_find_keyframes(_p(corr), F, tile_map_size, _p(kf))
    return kf, n


def tk_plan(pal, col):
    """DeviseBestMixingPlanThomasKnoll (main.pas:1828-1875): the luma-sorted 64-entry list for one colour."""
    pal = np.ascontiguousarray(pal, np.int32)
    out = np.zeros(64, np.uint8)
    lib().or_tk_plan(_p(pal), pal.size, int(np.int32(col)), _p(out))
    return out


def dither_tiles_tk(rgb, pal_of, palettes):
    """FinishDitherTiles per tile (DitherTile, Thomas Knoll + PrepareTileMirrors): (palpix, hm, vm)."""
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    palettes = np.ascontiguousarray(palettes, np.int32)
    n = rgb.shape[0]
    palpix = np.zeros((n, 64), np.uint8)
    hm = np.zeros(n, np.uint8)
    vm = np.zeros(n, np.uint8)
    lib().or_dither_tiles_tk(n, _p(rgb), _p(np.ascontiguousarray(pal_of, np.int32)), _p(palettes),
                             palettes.shape[1], _p(palpix), _p(hm), _p(vm))
    return palpix, hm, vm


def yl_plan(pal, col, mixed):
    """DeviseBestMixingPlanYliluoma (main.pas:1573-1826, the ASM_DBMP form): the luma-sorted list for one colour."""
    pal = np.ascontiguousarray(pal, np.int32)
    out = np.zeros(256, np.uint8)
    n = lib().or_yl_plan(_p(pal), pal.size, int(mixed), int(np.int32(col)), _p(out))
    return out[:n]


def dither_tiles_yl(rgb, pal_of, palettes, mixed):
    """FinishDitherTiles per tile with Yliluoma mixing (chkUseTK off) + PrepareTileMirrors: (palpix, hm, vm)."""
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    palettes = np.ascontiguousarray(palettes, np.int32)
    n = rgb.shape[0]
    palpix = np.zeros((n, 64), np.uint8)
    hm = np.zeros(n, np.uint8)
    vm = np.zeros(n, np.uint8)
    lib().or_dither_tiles_yl(n, _p(rgb), _p(np.ascontiguousarray(pal_of, np.int32)), _p(palettes),
                             palettes.shape[1], int(mixed), _p(palpix), _p(hm), _p(vm))
    return palpix, hm, vm


def ref_kmodes_lib():
    """The reference's own asm (kmodes.pas:316-596) if oracle/_ref was built here; else None."""
    if not os.path.exists(REF_LIB):
        return None
    r = ctypes.CDLL(REF_LIB)
    r.ref_get_min.restype = ctypes.c_int64
    return r


# ---- palette generation (palette.c): QuantizePalette with DLv3, CompareCMULHS, FinishQuantizePalette ----
def dl3quant(pixels, quant_to=16, bpc=7):
    """dl3quant over pixels [n][3] u8 (R, G, B): (palette [quant_to] 0x00BBGGRR, histogram colour count)."""
    px = np.ascontiguousarray(pixels, np.uint8).reshape(-1, 3)
    out = np.zeros(quant_to, np.int32)
    h = lib().or_dl3quant(_p(px), ctypes.c_long(px.shape[0]), quant_to, bpc, _p(out))
    return out, int(h)


def rgb_to_hsv(col):
    h, s, v = ctypes.c_uint8(), ctypes.c_uint8(), ctypes.c_uint8()
    lib().or_rgb_to_hsv(int(np.int32(col)), ctypes.byref(h), ctypes.byref(s), ctypes.byref(v))
    return h.value, s.value, v.value


def sort_cmulhs(cols):
    cols = np.ascontiguousarray(cols, np.int32)
    out = np.zeros_like(cols)
    lib().or_sort_cmulhs(_p(cols), cols.size, _p(out))
    return out


def quantize_palettes(rgb, pal_of, n_palettes, palsize=16, bpc=7, active=None, threads=None):
    """QuantizePalette for every palette of one keyframe: rgb [n][64] (0x00BBGGRR), pal_of [n] ->
    (palettes [P][palsize], use_count [P], histogram colour counts [P])."""
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    pal_of = np.ascontiguousarray(pal_of, np.int32)
    act = None if active is None else np.ascontiguousarray(active, np.uint8)
    pal = np.zeros((n_palettes, palsize), np.int32)
    uc = np.zeros(n_palettes, np.int32)
    hist = np.zeros(n_palettes, np.int32)
    lib().or_quantize_palettes(_p(rgb), _p(pal_of), _p(act), ctypes.c_long(rgb.shape[0]), n_palettes, palsize, bpc,
                               _p(pal), _p(uc), _p(hist), threads or _threads())
    return pal, uc, hist


def finish_quantize_order(use_count):
    """FinishQuantizePalette's order: lut[old palette] = new palette index."""
    uc = np.ascontiguousarray(use_count, np.int32)
    lut = np.zeros(uc.size, np.int32)
    lib().or_finish_quantize_order(_p(uc), uc.size, _p(lut))
    return lut


# ---- the Dither step's descriptors + k-means (PrepareDitherTiles restated; yakmo unpinned) ----
OR_LAB = 4


def psyv_lab_batch(rgb, gamma=-1, use_wavelets=True):
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    out = np.zeros((rgb.shape[0], 192), np.float64)
    lib().or_psyv_batch(rgb.shape[0], _p(rgb), None, None, None, None, OR_LAB | (2 if use_wavelets else 0), gamma,
                        _p(out))
    return out


def kmeans(X, k, max_iter=0x7fffffff, seed=0, threads=None):
    X = np.ascontiguousarray(X, np.float64)
    n, d = X.shape
    labels = np.zeros(n, np.int32)
    cent = np.zeros((k, d), np.float64)
    it = lib().or_kmeans(_p(X), ctypes.c_long(n), d, k, max_iter, ctypes.c_uint32(seed), _p(labels), _p(cent),
                         threads or _threads())
    return labels, cent, int(it)


def prepare_dither_tiles(rgb, n_palettes, gamma=-1, use_wavelets=True, max_iter=0x7fffffff, seed=0):
    rgb = np.ascontiguousarray(rgb, np.int32).reshape(-1, 64)
    if rgb.shape[0] <= 1 or n_palettes <= 1:
        return np.zeros(rgb.shape[0], np.int32), np.zeros((n_palettes, 192)), 0
    return kmeans(psyv_lab_batch(rgb, gamma, use_wavelets), n_palettes, max_iter, seed)


def generate_palettes(frames, kf_start, n_palettes, palsize=16, gamma=-1, use_wavelets=True, bpc=7):
    """btnDitherClick's palette half (main.pas:886-907) on the CPU restatement (see tiler_amd.palette)."""
    frames = np.ascontiguousarray(frames, np.int32)
    F, Q = frames.shape[:2]
    kf_start = np.asarray(kf_start, np.int64)
    KF, P = kf_start.size - 1, n_palettes
    pal = np.zeros((KF, P, palsize), np.int32)
    cent = np.zeros((KF, P, 192))
    dith = np.zeros(F * Q, np.int32)
    ucs = np.zeros((KF, P), np.int32)
    for k in range(KF):
        f0, f1 = int(kf_start[k]), int(kf_start[k + 1])
        tiles = frames[f0:f1].reshape(-1, 64)
        lab, c, _ = prepare_dither_tiles(tiles, P, gamma, use_wavelets)
        p, uc, _ = quantize_palettes(tiles, lab, P, palsize, bpc)
        lut = finish_quantize_order(uc)
        pal[k][lut] = p
        cent[k][lut] = c
        dith[f0 * Q:f1 * Q] = lut[lab]
        ucs[k][lut] = uc
    return pal, cent, dith, ucs

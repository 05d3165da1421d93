"""Python mirror of the reference's ANN usage (extern.pas:63-67 -> libANN.so).

`KDTree` keeps the reference call shape (create over rows, search / search_multi per query) and adds
the batched and HBM-resident forms the MI355X path is built around.  Every call runs on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import SearchStats, TilerError, check, load

FLT_MAX = np.float32(3.4028234663852886e38)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


ANN_KD_STD = 0            # TANNsplitRule (extern.pas:21-28): the reference's rule, ANN's tie order
SPLIT_INDEX_ORDER = 100   # extension: no kd-tree, equal distances resolve to the lowest index


class KDTree:
    """ann_kdtree_create(pa, n, dd, bs=1, split=ANN_KD_STD) ... ann_kdtree_destroy.

    split = ANN_KD_STD builds ANN's kd-tree so that ties come out as the reference's search returns them;
    split = SPLIT_INDEX_ORDER skips it (ties to the lowest index)."""

    def __init__(self, data=None, *, dev_ptr: int | None = None, n: int | None = None, dd: int | None = None,
                 stream: int = 0, bs: int = 1, split: int = ANN_KD_STD):
        lib = load()
        self._lib = lib
        if dev_ptr is not None:
            self.n, self.dd = int(n), int(dd)
            h = lib.ann_kdtree_create_dev_ex(ctypes.c_void_p(dev_ptr), self.n, self.dd, bs, split,
                                             ctypes.c_void_p(stream))
        else:
            data = np.ascontiguousarray(data, dtype=np.float32)
            if data.ndim != 2:
                raise ValueError("dataset must be [n, dd]")
            self.n, self.dd = data.shape
            self._rows = data
            # the float** row table (ANNpointArray) as one uint64 array: a per-row ctypes loop cost ~0.2 s at 262k rows
            rowp = np.uint64(data.ctypes.data) + np.arange(max(1, self.n), dtype=np.uint64) * np.uint64(4 * self.dd)
            self._rowp = rowp
            h = lib.ann_kdtree_create(rowp.ctypes.data_as(ctypes.POINTER(ctypes.POINTER(ctypes.c_float))), self.n,
                                      self.dd, bs, split)
        if not h:
            raise TilerError("ann_kdtree_create failed: " + lib.tiler_last_error().decode())
        self.handle = h

    @classmethod
    def adopt(cls, handle: int, n: int, dd: int) -> "KDTree":
        """Wrap a handle made by another entry point (tiler_prepare_frame_tiling_dev); destroyed on close."""
        if not handle:
            raise TilerError("null ann_kdtree handle: " + load().tiler_last_error().decode())
        t = cls.__new__(cls)
        t._lib = load()
        t.n, t.dd = int(n), int(dd)
        t.handle = handle
        return t

    def close(self):
        if getattr(self, "handle", None):
            self._lib.ann_kdtree_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- reference-shaped single-query calls (main.pas:4027, 3830) --
    def search(self, q, eps: float = 0.0):
        q = np.ascontiguousarray(q, dtype=np.float32)
        err = np.zeros(1, np.float32)
        idx = self._lib.ann_kdtree_search(self.handle, _ptr(q), eps, _ptr(err))
        check(idx if idx >= 0 or self.n == 0 else -1, "ann_kdtree_search")
        return int(idx), float(err[0])

    def pri_search(self, q, eps: float = 0.0):
        """ann_kdtree_pri_search (extern.pas:66): annkPriSearch's answer, its own tie order"""
        q = np.ascontiguousarray(q, dtype=np.float32)
        err = np.zeros(1, np.float32)
        idx = self._lib.ann_kdtree_pri_search(self.handle, _ptr(q), eps, _ptr(err))
        check(idx if idx >= 0 or self.n == 0 else -1, "ann_kdtree_pri_search")
        return int(idx), float(err[0])

    def search_multi(self, q, cnt: int, eps: float = 0.0):
        q = np.ascontiguousarray(q, dtype=np.float32)
        idxs = np.zeros(cnt, np.int32)
        errs = np.zeros(cnt, np.float32)
        check(self._lib.ann_kdtree_search_multi(self.handle, _ptr(idxs), _ptr(errs), cnt, _ptr(q), eps),
              "ann_kdtree_search_multi")
        return idxs, errs

    # -- batched --
    def search_batch(self, qs, k: int = 1, eps: float = 0.0):
        qs = np.ascontiguousarray(qs, dtype=np.float32).reshape(-1, self.dd)
        nq = qs.shape[0]
        idx = np.zeros((nq, k), np.int32)
        err = np.zeros((nq, k), np.float32)
        check(self._lib.ann_kdtree_search_multi_batch(self.handle, _ptr(qs), nq, k, eps, _ptr(idx), _ptr(err)),
              "ann_kdtree_search_multi_batch")
        return (idx[:, 0], err[:, 0]) if k == 1 else (idx, err)

    def pri_search_batch(self, qs, eps: float = 0.0):
        qs = np.ascontiguousarray(qs, dtype=np.float32).reshape(-1, self.dd)
        nq = qs.shape[0]
        idx = np.zeros(nq, np.int32)
        err = np.zeros(nq, np.float32)
        check(self._lib.ann_kdtree_pri_search_batch(self.handle, _ptr(qs), nq, eps, _ptr(idx), _ptr(err)),
              "ann_kdtree_pri_search_batch")
        return idx, err

    def search_batch_dev(self, q_ptr: int, nq: int, k: int, idx_ptr: int, err_ptr: int, stream: int = 0):
        check(self._lib.ann_kdtree_search_batch_dev(self.handle, ctypes.c_void_p(q_ptr), nq, k,
                                                    ctypes.c_void_p(idx_ptr), ctypes.c_void_p(err_ptr),
                                                    ctypes.c_void_p(stream)), "ann_kdtree_search_batch_dev")

    def stats(self) -> dict:
        s = SearchStats()
        check(self._lib.ann_kdtree_get_stats(self.handle, ctypes.byref(s)), "ann_kdtree_get_stats")
        return {"queries": s.queries, "fallback_queries": s.fallback_queries,
                "exhaustive_queries": s.exhaustive_queries, "exact_integer": s.exact_integer, "splits": s.splits,
                "orbit_groups": s.orbit_groups, "orbit_search": s.orbit_search, "orbit_ksteps": s.orbit_ksteps,
                "orbit_expansions": s.orbit_expansions, "orbit_rescored": s.orbit_rescored,
                "tie_order": s.tie_order, "kd_levels": s.kd_levels, "kd_build_ms": round(s.kd_build_ms, 3),
                "kd_replayed": s.kd_replayed, "flat_queries": s.flat_queries}

    def combine_stats(self) -> dict:
        """Coalescing of concurrent single-query calls on this handle (tiler_combine_stats)."""
        c, b, m = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
        check(self._lib.tiler_combine_stats(self.handle, ctypes.byref(c), ctypes.byref(b), ctypes.byref(m)),
              "tiler_combine_stats")
        return {"calls": c.value, "batches": b.value, "max_batch": m.value}

    def maps(self):
        """The TRTo* maps of the handle (tiler_ft_get_maps): (tile_of, pal_of, attrs) per dataset row."""
        t = np.zeros(max(self.n, 1), np.int32)
        p = np.zeros(max(self.n, 1), np.int32)
        a = np.zeros(max(self.n, 1), np.uint8)
        check(self._lib.tiler_ft_get_maps(self.handle, _ptr(t), _ptr(p), _ptr(a)), "tiler_ft_get_maps")
        return t[:self.n], p[:self.n], a[:self.n]

    def device(self) -> int:
        """The device the handle lives on (tiler_kdtree_device)."""
        return check(self._lib.tiler_kdtree_device(self.handle), "tiler_kdtree_device")

    def replicate(self, device: int = -1):
        """Copy the index to `device` now (-1 = every bound device; tiler_kdtree_replicate)."""
        check(self._lib.tiler_kdtree_replicate(self.handle, device), "tiler_kdtree_replicate")

    def positions(self) -> np.ndarray:
        """Leaf position of every point in ANN's kd-tree (tiler_kdtree_positions)."""
        pos = np.zeros(self.n, np.int32)
        if self.n:
            check(self._lib.tiler_kdtree_positions(self.handle, _ptr(pos)), "tiler_kdtree_positions")
        return pos

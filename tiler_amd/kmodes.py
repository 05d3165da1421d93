"""GlobalTiling K-Modes (TKModes.ComputeKModes kmodes.pas:917-1060) on libANN.so."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load


def compute_kmodes(X, k: int, start_point: int, n_modalities: int = 16):
    """ComputeKModes(X, k, ANumInit=-start_point, modalities): returns (labels, centroids, n_iter, cost)."""
    lib = load()
    X = np.ascontiguousarray(X, np.uint8)
    n, a = X.shape
    labels = np.zeros(n, np.int32)
    cent = np.zeros((k, a), np.uint8)
    it = ctypes.c_int(0)
    cost = ctypes.c_uint64(0)
    v = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    check(lib.tiler_kmodes_compute(v(X), n, a, k, start_point, n_modalities, v(labels), v(cent), ctypes.byref(it),
                                   ctypes.byref(cost)), "tiler_kmodes_compute")
    return labels, cent, it.value, cost.value

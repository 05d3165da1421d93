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


def compute_kmodes_batch(X, bin_off, k, start, n_modalities: int = 16):
    """All palette bins at once (tiler_kmodes_batch): X [N][80] with bin b = rows bin_off[b]:bin_off[b+1].
    Returns (labels [N] bin-local, centroids [sum k][80], n_iter [nb], cost [nb])."""
    lib = load()
    X = np.ascontiguousarray(X, np.uint8)
    bin_off = np.ascontiguousarray(bin_off, np.int32)
    k = np.ascontiguousarray(k, np.int32)
    start = np.ascontiguousarray(start, np.int32)
    nb = k.size
    labels = np.zeros(X.shape[0], np.int32)
    cent = np.zeros((int(k.sum()), X.shape[1]), np.uint8)
    it = np.zeros(nb, np.int32)
    cost = np.zeros(nb, np.uint64)
    v = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    check(lib.tiler_kmodes_batch(v(X), v(bin_off), nb, v(k), v(start), n_modalities, v(labels), v(cent), v(it),
                                 v(cost)), "tiler_kmodes_batch")
    return labels, cent, it, cost


def medoids_batch(X, bin_off, k, labels, centroids):
    """tiler_kmodes_medoids_batch: per cluster (bin after bin) the bin-local medoid row and member count."""
    lib = load()
    X = np.ascontiguousarray(X, np.uint8)
    k = np.ascontiguousarray(k, np.int32)
    K = int(k.sum())
    medoid = np.zeros(K, np.int32)
    counts = np.zeros(K, np.int32)
    v = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    check(lib.tiler_kmodes_medoids_batch(v(X), v(np.ascontiguousarray(bin_off, np.int32)), k.size, v(k),
                                         v(np.ascontiguousarray(labels, np.int32)),
                                         v(np.ascontiguousarray(centroids, np.uint8)), v(medoid), v(counts)),
          "tiler_kmodes_medoids_batch")
    return medoid, counts

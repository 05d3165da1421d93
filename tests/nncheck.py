"""Shared GPU-vs-oracle NN checks: every search is compared under BOTH tie rules.

* default handle (split = ANN_KD_STD, the reference's ann_kdtree_create call, main.pas:3779,3961) against
  oracle/ann_kdtree.c, the ANN 1.1.2 kd-tree search restated (the reference's first-found tie order);
* split = TILER_SPLIT_INDEX_ORDER (100) against the exhaustive lowest-index scan (oracle/tiler_oracle.c).
Indices and fp32 distances must agree bit for bit.
"""
import numpy as np

INDEX_ORDER = 100


SCAN_DEFAULT = (64, 16)  # tiler_set_scan_limits defaults (include/tiler_ann.h)


def check_nn(gpu, oracle, data, qs, k=1, bs=1):
    """k nearest neighbours of qs under both tie rules; returns the kd-order handle's stats.  A batch small enough for
    the exhaustive small-batch scan is searched twice under the kd order: by that scan and, with it disabled, by the
    MFMA shortlist and its tiers (whose stats are returned); both must equal the oracle."""
    data = np.ascontiguousarray(data, np.float32)
    qs = np.ascontiguousarray(qs, np.float32).reshape(-1, data.shape[1])
    lib = gpu.load()
    small = qs.shape[0] <= (SCAN_DEFAULT[0] if k == 1 else SCAN_DEFAULT[1] if k <= 8 else 0)
    runs = []
    try:
        for limits in ((SCAN_DEFAULT, (0, 0)) if small else (SCAN_DEFAULT,)):
            assert lib.tiler_set_scan_limits(*limits) == 0
            with gpu.KDTree(data, bs=bs) as kdt:
                gi, ge = kdt.search_batch(qs, k=k)
                runs.append((gi, ge, kdt.stats()))
    finally:
        lib.tiler_set_scan_limits(*SCAN_DEFAULT)
    okd = oracle.KDTree(data, bs=bs)
    oi, oe = okd.search_batch(qs, k=k)
    okd.close()
    for gi, ge, st in runs:
        assert np.array_equal(ge.view(np.uint32), oe.view(np.uint32)), "kd order: distance mismatch"
        bad = np.nonzero(np.any((gi != oi).reshape(qs.shape[0], -1), axis=1))[0]
        assert bad.size == 0, f"kd order: {bad.size} of {qs.shape[0]} queries differ (first {bad[:8]})"
    with gpu.KDTree(data, split=INDEX_ORDER) as kdt:
        gi2, ge2 = kdt.search_batch(qs, k=k)
        assert kdt.stats()["tie_order"] == 1
    if k == 1:
        oi2, oe2 = oracle.nn_batch(data, qs)
    else:
        res = [oracle.knn(data, q, k) for q in qs]
        oi2 = np.stack([r[0] for r in res])
        oe2 = np.stack([r[1] for r in res])
    assert np.array_equal(ge2.view(np.uint32), oe2.view(np.uint32)), "index order: distance mismatch"
    assert np.array_equal(gi2, oi2), f"index order: {np.count_nonzero(gi2 != oi2)} index mismatches"
    return st

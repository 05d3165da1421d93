"""CPU check of the derivation behind kd_median_big_kernel (tiler_amd/csrc/kdtree.hip): ANN 1.1.2's annMedianSplit
(kd_util.cpp; the DLL's 0x180015cf0) made data-parallel.  The sequential Hoare loop swaps
exactly the pairs (L_j, R_j) of the ORIGINAL array's left stoppers (key >= c in (l, r], ascending) and right stoppers
(key <= c in [l, r), descending) with L_j < R_j, and stops at k = R_J or max(R_J, L_{J-1}); each lane decides
"L_j < R_j" from the ranks alone (right stoppers above L_j >= j).  This emulates the kernel's rank arithmetic step by
step and compares the permutation, the split point and the cut value with the sequential loop on random arrays with
many equal keys (the case that decides which equal keys go LO).  The GPU tree itself is checked against
oracle/ann_kdtree.c in tests/test_gpu_orbit.py."""
import numpy as np


def _sequential(key, idx, n_lo):
    key, idx = key.copy(), idx.copy()

    def sw(a, b):
        key[a], key[b] = key[b], key[a]
        idx[a], idx[b] = idx[b], idx[a]

    l, r = 0, len(key) - 1
    while l < r:
        i = (r + l) // 2
        if key[i] > key[r]:
            sw(i, r)
        sw(l, i)
        c, i, k = key[l], l, r
        while True:
            i += 1
            while key[i] < c:
                i += 1
            k -= 1
            while key[k] > c:
                k -= 1
            if i < k:
                sw(i, k)
            else:
                break
        sw(l, k)
        if k > n_lo:
            r = k - 1
        elif k < n_lo:
            l = k + 1
        else:
            break
    if n_lo > 0:
        m = 0
        for i in range(1, n_lo):
            if key[i] > key[m]:
                m = i
        sw(n_lo - 1, m)
    return key, idx, np.float32((np.float64(np.float32(key[n_lo - 1] + key[n_lo]))) / 2.0)


def _parallel(key, idx, n_lo):
    key, idx = key.copy(), idx.copy()

    def sw(a, b):
        key[a], key[b] = key[b], key[a]
        idx[a], idx[b] = idx[b], idx[a]

    l, r = 0, len(key) - 1
    while l < r:
        i = (r + l) // 2
        if key[i] > key[r]:
            sw(i, r)
        sw(l, i)
        c = key[l]
        p = np.arange(l, r + 1)
        v = key[l:r + 1]
        isl = (p > l) & ~(v < c)   # where `while key[++i] < c` stops (NaN keys / a NaN pivot stop it too)
        isr = (p < r) & ~(v > c)   # where `while key[--k] > c` stops
        tot_r = int(isr.sum())
        jl = np.cumsum(isl)                  # rank from the left (1-based) at left stoppers
        rb = np.cumsum(isr) - isr            # right stoppers below p
        lpos = p[isl]
        rpos = np.empty(tot_r, np.int64)
        rpos[(tot_r - rb - 1)[isr]] = p[isr]  # index = rank from the right - 1
        swapped = isl & ((tot_r - rb - isr) >= jl)
        npair = int(swapped.sum())
        assert swapped[isl][:npair].all() and not swapped[isl][npair:].any()  # a prefix of the pairs
        for j in range(npair):
            sw(lpos[j], rpos[j])
        k = rpos[npair]
        if npair > 0:
            k = max(k, lpos[npair - 1])
        sw(l, k)
        if k > n_lo:
            r = k - 1
        elif k < n_lo:
            l = k + 1
        else:
            break
    if n_lo > 0:  # the first maximum, NaN keys skipped; a NaN key[0] is never replaced (kd_median_big_kernel)
        head = key[:n_lo]
        ok = ~np.isnan(head)
        m = 0 if (np.isnan(head[0]) or not ok.any()) else int(np.flatnonzero(ok)[np.argmax(head[ok])])
        sw(n_lo - 1, m)
    return key, idx, np.float32((np.float64(np.float32(key[n_lo - 1] + key[n_lo]))) / 2.0)


def _same(a, b):
    return (np.array_equal(a[0], b[0], equal_nan=True) and np.array_equal(a[1], b[1]) and
            (a[2] == b[2] or (np.isnan(a[2]) and np.isnan(b[2]))))


def test_parallel_hoare_with_nan_and_inf_keys():
    """Non-finite keys: NaN stops both scans in the sequential loop (its `<` / `>` tests fail), a NaN
    pivot makes every position a stopper; the ranked form must make the same swaps and never index past the
    stoppers it counted.  +-inf are ordinary ordered keys."""
    rng = np.random.default_rng(7)
    with np.errstate(invalid="ignore"):
        for t in range(1500):
            n = int(rng.integers(2, 300))
            key = rng.integers(0, int(rng.integers(1, 9)), n).astype(np.float32)
            frac = [0.02, 0.2, 0.6, 1.0][t % 4]
            key[rng.random(n) < frac] = np.nan
            if t % 5 == 0:
                key[rng.random(n) < 0.1] = np.inf
                key[rng.random(n) < 0.1] = -np.inf
            if t % 7 == 0:
                key[(n - 1) // 2] = np.nan  # the first pivot
            idx = np.arange(n, dtype=np.int64)
            assert _same(_sequential(key, idx, n // 2), _parallel(key, idx, n // 2)), (t, n)


def test_parallel_hoare_ranking_equals_annmediansplit():
    rng = np.random.default_rng(20261017)
    for t in range(1500):
        n = int(rng.integers(2, 400))
        if t % 3 == 0:
            key = rng.integers(0, int(rng.integers(1, 12)), n).astype(np.float32)  # heavy ties
        elif t % 3 == 1:
            key = rng.standard_normal(n).astype(np.float32)
        else:
            key = np.sort(rng.integers(0, 5, n)).astype(np.float32)[::int(rng.choice([-1, 1]))].copy()
        idx = np.arange(n, dtype=np.int64)
        a, b = _sequential(key, idx, n // 2), _parallel(key, idx, n // 2)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2], (t, n)

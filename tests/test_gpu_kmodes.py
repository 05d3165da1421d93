"""GPU parity of K-Modes against the CPU restatement (pinned to the reference asm): labels, centroids,
iteration count and cost bit-exact, including empty-cluster rescues (Delphi LCG) and ties."""
import os

import numpy as np
import pytest

from tiler_amd.kmodes import compute_kmodes

pytestmark = pytest.mark.gpu


def _dataset(rng, n, protos, noise):
    """80-byte rows as WriteTileDatasetLine makes them (64 palette indices + 16 zone flags)."""
    P = rng.integers(0, 16, (protos, 64)).astype(np.uint8)
    X = P[rng.integers(0, protos, n)].copy()
    flip = rng.random(X.shape) < noise
    X[flip] = rng.integers(0, 16, int(flip.sum()))
    acc = np.stack([(X == z).sum(1) for z in range(16)], 1)
    return np.concatenate([X, (acc > 1).astype(np.uint8)], 1)


@pytest.mark.parametrize("n,k,protos,noise", [(500, 20, 30, 0.1), (2500, 97, 200, 0.15), (3000, 400, 60, 0.05),
                                              (1200, 300, 1200, 0.5)])
def test_kmodes_bit_exact(gpu, oracle, n, k, protos, noise):
    rng = np.random.default_rng(n + k)
    X = _dataset(rng, n, protos, noise)
    start = int(np.argmin(X.astype(np.int64).sum(1)[::-1]))
    start = n - 1 - start  # last row with minimal byte sum (DoGlobalTiling main.pas:4303-4308)
    gl, gc, gi, gcost = compute_kmodes(X, k, start)
    ol, oc, oi, ocost = oracle.kmodes(X, k, start)
    assert (gi, gcost) == (oi, ocost)
    assert np.array_equal(gl, ol) and np.array_equal(gc, oc)


def test_kmodes_batch_ff_fallback_bit_exact(gpu, oracle):
    """the recovery path of the persistent farthest-first (a grid barrier that gives up sets the fail word,
    every workgroup leaves, the host re-initialises the state and re-runs the rounds one launch each), forced through
    tiler_debug_kmodes_ff_fallback: a batch of bins must give the restatement's labels, centroids, iterations and cost,
    and the same outputs as the persistent path."""
    from tiler_amd.kmodes import compute_kmodes_batch
    rng = np.random.default_rng(77)
    sizes, ks = [2500, 1800, 900, 400], [120, 95, 40, 17]
    X = np.concatenate([_dataset(rng, n, 150, 0.12) for n in sizes])
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    k = np.array(ks, np.int32)
    starts = np.array([int(np.argmin(X[off[b]:off[b + 1]].astype(np.int64).sum(1))) for b in range(len(sizes))], np.int32)
    import ctypes
    lib = gpu.load()
    assert lib.tiler_debug_kmodes_ff_fallback(1) == 0
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    try:
        fl, fc, fi, fcost = compute_kmodes_batch(X, off, k, starts)
    finally:
        lib.tiler_debug_kmodes_ff_fallback(0)
        lib.tiler_timing_enable(0)
    n_init = ctypes.c_int(0)
    lib.tiler_timing_get(b"kmodes_init", ctypes.byref(n_init))
    assert n_init.value == 2  # the persistent launch, then the recovery's per-launch rounds
    pl, pc, pi, pcost = compute_kmodes_batch(X, off, k, starts)
    assert np.array_equal(fl, pl) and np.array_equal(fc, pc) and np.array_equal(fi, pi) and np.array_equal(fcost, pcost)
    koff = np.concatenate([[0], np.cumsum(ks)])
    for b in range(len(sizes)):
        ol, oc, oi, ocost = oracle.kmodes(X[off[b]:off[b + 1]], ks[b], int(starts[b]))
        assert (int(fi[b]), int(fcost[b])) == (oi, ocost), b
        assert np.array_equal(fl[off[b]:off[b + 1]], ol) and np.array_equal(fc[koff[b]:koff[b + 1]], oc), b


@pytest.mark.parametrize("modalities,vmax", [(64, 64), (200, 200), (8, 8)])
def test_kmodes_other_modalities(gpu, oracle, modalities, vmax):
    """Byte values beyond 15 (64 / 200 modalities) run the general assignment (kmb_assign: the asm's int8 |r - x|
    and the W0 / W4 wrap do matter there) and the general mode-rule walk; 8 modalities the <= 16 forms."""
    rng = np.random.default_rng(modalities)
    protos = rng.integers(0, vmax, (80, 80)).astype(np.uint8)
    X = protos[rng.integers(0, 80, 1500)].copy()
    flip = rng.random(X.shape) < 0.2
    X[flip] = rng.integers(0, vmax, int(flip.sum()))
    gl, gc, gi, gcost = compute_kmodes(X, 60, 3, n_modalities=modalities)
    ol, oc, oi, ocost = oracle.kmodes(X, 60, 3, modalities=modalities)
    assert (gi, gcost) == (oi, ocost)
    assert np.array_equal(gl, ol) and np.array_equal(gc, oc)


def test_kmodes_more_clusters_than_clash_table(gpu, oracle):
    """K = 8,500 > the move pass's 8,192-bucket clash table (kmodes.hip KM_CLASH_TAB): clusters share buckets, which
    may only end a group of concurrent moves early; labels, centroids, iterations and cost stay bit-exact."""
    rng = np.random.default_rng(8500)
    X = _dataset(rng, 20000, 2000, 0.3)  # 5 iterations with moves (about 10 s of the oracle on 8 threads)
    start = 20000 - 1 - int(np.argmin(X.astype(np.int64).sum(1)[::-1]))
    gl, gc, gi, gcost = compute_kmodes(X, 8500, start)
    ol, oc, oi, ocost = oracle.kmodes(X, 8500, start, threads=_oracle_threads())
    assert (gi, gcost) == (oi, ocost)
    assert np.array_equal(gl, ol) and np.array_equal(gc, oc)


def test_kmodes_duplicates_force_rescue(gpu, oracle):
    rng = np.random.default_rng(77)
    X = _dataset(rng, 800, 5, 0.0)  # 5 distinct rows only: farthest-first picks duplicates, clusters empty
    X[::7, 3] = 9
    gl, gc, gi, gcost = compute_kmodes(X, 40, 0)
    ol, oc, oi, ocost = oracle.kmodes(X, 40, 0)
    assert (gi, gcost) == (oi, ocost) and np.array_equal(gl, ol) and np.array_equal(gc, oc)


def test_kmodes_batch_matches_per_bin(gpu, oracle):
    """tiler_kmodes_batch over bins of different sizes / K (the GlobalTiling call shape, main.pas:4339):
    every bin bit-identical to its own ComputeKModes run."""
    from tiler_amd.kmodes import compute_kmodes_batch, medoids_batch
    rng = np.random.default_rng(5)
    sizes = [1500, 37, 960, 961, 400, 1, 2200]
    ks = [90, 37, 50, 200, 12, 1, 300]
    Xs = [_dataset(rng, n, max(2, n // 10), 0.1) for n in sizes]
    X = np.concatenate(Xs)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    starts = [int(n - 1 - np.argmin(x.astype(np.int64).sum(1)[::-1])) for n, x in zip(sizes, Xs)]
    labels, cent, iters, costs = compute_kmodes_batch(X, off, ks, starts)
    koff = np.concatenate([[0], np.cumsum(ks)])
    med, cnt = medoids_batch(X, off, ks, labels, cent)
    for b, (x, k, st) in enumerate(zip(Xs, ks, starts)):
        ol, oc, oi, ocost = oracle.kmodes(x, k, st)
        assert (int(iters[b]), int(costs[b])) == (oi, ocost), b
        assert np.array_equal(labels[off[b]:off[b + 1]], ol), b
        assert np.array_equal(cent[koff[b]:koff[b + 1]], oc), b
        from tiler_amd.global_tiling import kmodes_medoids
        m1, c1 = kmodes_medoids(x, ol, oc)
        assert np.array_equal(med[koff[b]:koff[b + 1]], m1) and np.array_equal(cnt[koff[b]:koff[b + 1]], c1), b


def test_kmodes_batch_many_bins_host_list(gpu, oracle):
    """More active bins than the device work-list generator takes (kmodes.hip KM_GEN_MAXB = 4,096): the iteration's
    list is built on the host instead, and bins leave the active set at different iterations; 4,500 small bins, every
    one bit-identical to its own ComputeKModes run."""
    from tiler_amd.kmodes import compute_kmodes_batch
    rng = np.random.default_rng(4500)
    sizes = rng.integers(3, 13, 4500)
    ks = [int(rng.integers(1, n)) for n in sizes]
    Xs = [_dataset(rng, int(n), 3, 0.3) for n in sizes]
    X = np.concatenate(Xs)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    starts = [int(n - 1 - np.argmin(x.astype(np.int64).sum(1)[::-1])) for n, x in zip(sizes, Xs)]
    labels, cent, iters, costs = compute_kmodes_batch(X, off, ks, starts)
    koff = np.concatenate([[0], np.cumsum(ks)])
    assert len(set(int(i) for i in iters)) > 1  # the active set shrinks over the iterations
    for b, (x, k, st) in enumerate(zip(Xs, ks, starts)):
        ol, oc, oi, ocost = oracle.kmodes(x, k, st)
        assert (int(iters[b]), int(costs[b])) == (oi, ocost), b
        assert np.array_equal(labels[off[b]:off[b + 1]], ol), b
        assert np.array_equal(cent[koff[b]:koff[b + 1]], oc), b


def _oracle_threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 1


@pytest.mark.timeout(1200)
def test_kmodes_c4_full_batch(gpu, oracle):
    """BASELINE C4 at full size: 1,048,576 tiles (64k prototypes, 10 % perturbation, Zipf(1.1) bins over 128
    palettes, desired 65,536) through ONE tiler_kmodes_batch + medoid batch (the DoGlobalTiling call shape,
    main.pas:4339), then every bin of <= 10,000 rows (111 bins) and the FOUR LARGEST bins (236,865 / 110,181 /
    70,453 / 51,715 rows, K = 5,035 / 3,222 / 2,477 / 2,064: the critical path, where the grouped concurrent moves
    and the split assignment carry the most weight, kmodes.pas:845-915) checked against the CPU restatement
    (labels, centroids, iterations, cost, medoids; the oracle's distance loops on 16 host threads like the
    reference's TKModes threads; about two minutes of host time)."""
    from tiler_amd import global_tiling as gt
    from tiler_amd import synth
    tiles, dith = synth.globaltiling_workload(4, 1 << 20, n_palettes=128)
    plan = gt.plan_global_tiling(tiles, dith, 128, 65536)
    from tiler_amd.kmodes import compute_kmodes_batch, medoids_batch
    run = list(plan.run)
    X_all = np.ascontiguousarray(np.concatenate([plan.lines[plan.bins[p]] for p in run]))
    off = np.concatenate([[0], np.cumsum([plan.bins[p].size for p in run])]).astype(np.int32)
    ks = np.array([plan.k_per_bin[p] for p in run], np.int32)
    st = np.array([plan.starts[p] for p in run], np.int32)
    assert X_all.shape[0] == (1 << 20) - sum(plan.bins[p].size for p in range(128) if p not in run)
    g_labels, g_cent, g_it, g_cost = compute_kmodes_batch(X_all, off, ks, st)
    g_med, g_cnt = medoids_batch(X_all, off, ks, g_labels, g_cent)
    koff = np.concatenate([[0], np.cumsum(ks)])
    largest = sorted(range(len(run)), key=lambda b: -(off[b + 1] - off[b]))[:4]
    assert off[largest[0] + 1] - off[largest[0]] == 236865 and ks[largest[0]] == 5035
    check = [b for b in range(len(run)) if off[b + 1] - off[b] <= 10000] + largest
    assert len(check) >= 100
    th = _oracle_threads()
    for b in check:
        p = run[b]
        X = plan.lines[plan.bins[p]]
        k = int(ks[b])
        ol, oc, oi, ocost = oracle.kmodes(X, k, plan.starts[p], threads=th)
        labels = g_labels[off[b]:off[b + 1]]
        medoid, counts = g_med[koff[b]:koff[b + 1]], g_cnt[koff[b]:koff[b + 1]]
        assert (int(g_it[b]), int(g_cost[b])) == (oi, ocost), p
        assert np.array_equal(g_cent[koff[b]:koff[b + 1]], oc), p
        assert np.array_equal(labels, ol), p
        assert np.array_equal(counts, np.bincount(ol, minlength=k)), p
        for j in np.nonzero(counts)[0]:
            mem = np.nonzero(ol == j)[0]
            i, _ = oracle.km_get_min(X[mem], oc[j])  # GetMinMatchingDissim: ties -> last member
            assert medoid[j] == mem[i], (p, j)


@pytest.mark.timeout(1200)
def test_kmodes_c5_shaped_batch(gpu, oracle):
    """A C5-shaped GlobalTiling (BASELINE C5: the reduced tileset is 256k tiles): 4,194,304 tiles from 262,144
    prototypes over 128 Zipf bins, desired 262,144 clusters, in ONE tiler_kmodes_batch + medoid batch.  Every bin of
    <= 10,000 rows is checked against the restatement; for all bins the labels are in range, each non-empty
    cluster's medoid is one of its members, and the reported cost is the sum of the final snapshot distances that
    the labels imply (recomputed on the host for the checked bins)."""
    from tiler_amd import global_tiling as gt
    from tiler_amd import synth
    from tiler_amd.kmodes import compute_kmodes_batch, medoids_batch
    tiles, dith = synth.globaltiling_workload(5, 1 << 22, protos=1 << 18, n_palettes=128)
    plan = gt.plan_global_tiling(tiles, dith, 128, 1 << 18)
    run = list(plan.run)
    X_all = np.ascontiguousarray(np.concatenate([plan.lines[plan.bins[p]] for p in run]))
    off = np.concatenate([[0], np.cumsum([plan.bins[p].size for p in run])]).astype(np.int32)
    ks = np.array([plan.k_per_bin[p] for p in run], np.int32)
    st = np.array([plan.starts[p] for p in run], np.int32)
    assert 250000 <= int(ks.sum()) <= 270000, int(ks.sum())
    g_labels, g_cent, g_it, g_cost = compute_kmodes_batch(X_all, off, ks, st)
    g_med, g_cnt = medoids_batch(X_all, off, ks, g_labels, g_cent)
    koff = np.concatenate([[0], np.cumsum(ks)])
    for b in range(len(run)):
        lab = g_labels[off[b]:off[b + 1]]
        assert lab.min() >= 0 and lab.max() < ks[b], b
        cnt = g_cnt[koff[b]:koff[b + 1]]
        assert np.array_equal(cnt, np.bincount(lab, minlength=int(ks[b]))), b
        med = g_med[koff[b]:koff[b + 1]]
        nz = cnt > 0
        assert np.array_equal(lab[med[nz]], np.nonzero(nz)[0]), b  # each medoid belongs to its cluster
    th = _oracle_threads()
    small = [b for b in range(len(run)) if off[b + 1] - off[b] <= 10000]
    assert len(small) >= 60
    for b in small:
        p = run[b]
        ol, oc, oi, ocost = oracle.kmodes(plan.lines[plan.bins[p]], int(ks[b]), plan.starts[p], threads=th)
        assert (int(g_it[b]), int(g_cost[b])) == (oi, ocost), p
        assert np.array_equal(g_labels[off[b]:off[b + 1]], ol), p
        assert np.array_equal(g_cent[koff[b]:koff[b + 1]], oc), p

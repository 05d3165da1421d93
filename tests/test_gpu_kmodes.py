"""GPU parity of K-Modes against the CPU restatement (pinned to the reference asm): labels, centroids,
iteration count and cost bit-exact, including empty-cluster rescues (Delphi LCG) and ties."""
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

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

"""The small-batch exact scan (the reference's per-tile ann_kdtree_search calls, coalesced by the library;
SURVEY.md 8(b); nn_scan_small_kernel + nn_scan_merge_kernel), bit-exact against the restated ANN search and the
lowest-index scan (nncheck, which also runs each batch through the MFMA tiers): batches of 1..64 queries, a prefix of
equal dimensions with coarse-grid values and duplicated rows (ties in ANN's order), rows at +inf distance, rows of
4..36 dimensions, and more than 256 candidates per workgroup at the 1,024-split cap.  (Round 5 also measured a
partial-distance pruning of this scan against these tests: exact, but no faster on PsyV rows -- DESIGN.md section 4.)"""
import numpy as np
import pytest

from nncheck import check_nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nq", [1, 3, 16, 64])
def test_scan_small_random(gpu, oracle, nq):
    rng = np.random.default_rng(100 + nq)
    data = rng.standard_normal((5000, 192)).astype(np.float32)
    q = data[rng.choice(5000, nq, replace=False)] + rng.standard_normal((nq, 192)).astype(np.float32) * 0.3
    check_nn(gpu, oracle, data, q)


def test_scan_small_flat_prefix_and_ties(gpu, oracle):
    """The first 32 dimensions equal in every row (the prefix bounds nothing), values on a coarse grid (many equal
    distances), duplicated rows (ties resolved by the tie order)."""
    rng = np.random.default_rng(7)
    base = (rng.integers(0, 3, (3000, 128)) * 0.5).astype(np.float32)
    data = np.concatenate([np.full((3000, 32), 0.25, np.float32), base], axis=1)
    data = np.concatenate([data, data[:1500]])
    q = data[rng.choice(data.shape[0], 40, replace=False)]
    check_nn(gpu, oracle, data, q)


def test_scan_small_infinite_distances(gpu, oracle):
    """Rows whose squares overflow to +inf inside the prefix or after it (NaN rows are out: what ANN returns around a
    NaN distance depends on its visit order, test_gpu_edges::test_nonfinite_dataset_builds_and_searches)."""
    rng = np.random.default_rng(8)
    data = rng.standard_normal((4000, 64)).astype(np.float32)
    data[::97, 5] = 3e19            # +inf inside the prefix
    data[3::101, 50] = -3e19        # +inf after it
    data[7::89, :] = 3e19           # every term +inf
    q = rng.standard_normal((20, 64)).astype(np.float32)
    check_nn(gpu, oracle, data, q)


@pytest.mark.parametrize("d", [4, 32, 36])
def test_scan_small_short_rows(gpu, oracle, d):
    rng = np.random.default_rng(9 + d)
    data = rng.standard_normal((6000, d)).astype(np.float32)
    check_nn(gpu, oracle, data, rng.standard_normal((17, d)).astype(np.float32))


def test_scan_small_several_rounds_per_thread(gpu, oracle):
    """300,000 candidates: more than 256 per workgroup at the 1,024-split cap, so the bound carries over rounds."""
    rng = np.random.default_rng(10)
    data = rng.standard_normal((300000, 48)).astype(np.float32)
    q = data[rng.choice(300000, 9, replace=False)] + 0.05
    check_nn(gpu, oracle, data, q)

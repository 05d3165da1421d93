"""GPU parity of the kd-tree build (ANN 1.1.2 ANN_KD_STD via kdtree.hip) against the restated ANN
build (oracle/ann_kdtree.c): the leaf position of every point -- i.e. annMedianSplit's permutation at every node,
which decides which of several equal keys go LO -- on shapes that cross every build path (a whole tree inside one
subtree workgroup, subtree levels run by several waves per node, big levels split into spread chunks, dimensions
beyond the multi-wave partials), on tie-heavy data (few distinct values per dimension), and through a search whose
ties resolve in the tree's order."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rows(seed, n, dd, levels):
    rng = np.random.default_rng(seed)
    if levels:
        return (rng.integers(0, levels, (n, dd)) * 0.25).astype(np.float32)
    return rng.standard_normal((n, dd)).astype(np.float32)


@pytest.mark.parametrize("n,dd,levels,bs", [
    (1, 5, 0, 1), (2, 3, 0, 1), (3, 7, 3, 1), (17, 4, 2, 1), (700, 192, 0, 1), (1024, 64, 4, 1),
    (1025, 192, 3, 1), (5000, 3, 5, 1), (3000, 300, 3, 1), (70000, 64, 6, 1), (40000, 192, 0, 1), (9000, 16, 2, 4),
])
def test_kd_positions_match_ann(gpu, oracle, n, dd, levels, bs):
    rows = _rows(n * 7 + dd, n, dd, levels)
    with gpu.KDTree(rows, bs=bs) as kdt:
        pos = kdt.positions()
    okd = oracle.KDTree(rows, bs=bs)
    opos = okd.positions()
    okd.close()
    assert np.array_equal(pos, opos), f"leaf order differs at {np.count_nonzero(pos != opos)} points"


def test_kd_tie_order_search_matches_ann(gpu, oracle):
    """Duplicated rows: every query has several candidates at distance 0, and the answer is the copy ANN's search
    meets first -- decided by the build's permutation."""
    rng = np.random.default_rng(5)
    base = _rows(6, 6000, 48, 3)
    rows = np.concatenate([base, base[rng.permutation(6000)], base[:3000]])
    q = rows[rng.choice(rows.shape[0], 2000, replace=False)]
    with gpu.KDTree(rows) as kdt:
        gi, ge = kdt.search_batch(q)
    okd = oracle.KDTree(rows)
    oi, oe = okd.search_batch(q)
    okd.close()
    assert np.array_equal(gi, oi) and np.array_equal(ge, oe)

"""ann_kdtree_pri_search (extern.pas:66; ANN.dll 0x180003ef0 -> annkPriSearch 0x1800121a0, k = 1) on the GPU
(kd_pri_kernel: the priority search replayed, its heap in HBM) against the oracle's restatement
(or_kdtree_pri_search_batch, pinned by tests/test_ann_kdtree.py::test_oracle_pri_search_matches_python_restatement):
index and distance bits, eps = 0 and eps = 0.5, ANN_KD_STD trees with buckets of 1 and 4, on datasets full of exact
ties (integer rows, duplicated rows, a mirror-orbit tileset) and on PsyV rows."""
import numpy as np
import pytest

from tiler_amd import synth

pytestmark = pytest.mark.gpu


def _check(gpu, oracle, data, qs, eps, bs=1):
    data = np.ascontiguousarray(data, np.float32)
    qs = np.ascontiguousarray(qs, np.float32)
    with gpu.KDTree(data, bs=bs) as kdt:
        gi, ge = kdt.pri_search_batch(qs, eps)
        si, se = kdt.search_batch(qs)
        li, le = kdt.pri_search(qs[0], eps)  # the single-query entry point
    okd = oracle.KDTree(data, bs=bs)
    oi, oe = okd.pri_search_batch(qs, eps)
    okd.close()
    assert np.array_equal(ge.view(np.uint32), oe.view(np.uint32)), "pri search: distance mismatch"
    bad = np.nonzero(gi != oi)[0]
    assert bad.size == 0, f"pri search: {bad.size} of {len(qs)} indices differ (first {bad[:8]})"
    assert li == oi[0] and np.float32(le).view(np.uint32) == oe[0].view(np.uint32)
    if eps == 0.0:
        assert np.array_equal(ge, se)  # exact: the same minimum distance as annkSearch
    return int(np.count_nonzero(gi != si))


@pytest.mark.parametrize("eps", [0.0, 0.5])
@pytest.mark.parametrize("bs", [1, 4])
def test_pri_search_ties(gpu, oracle, eps, bs):
    rng = np.random.default_rng(40 + bs)
    ints = rng.integers(0, 3, (3000, 8)).astype(np.float32)
    base = rng.normal(0, 1, (700, 24)).astype(np.float32)
    dup = np.concatenate([base, base[::-1], base[:300]])
    differ = 0
    for data in (ints, dup):
        n = data.shape[0]
        qs = np.concatenate([data[rng.integers(0, n, 100)],
                             data[rng.integers(0, n, 100)] + rng.integers(-1, 2, (100, data.shape[1])),
                             rng.normal(0, 2, (56, data.shape[1]))]).astype(np.float32)
        differ += _check(gpu, oracle, data, qs, eps, bs)
    if eps == 0.0:
        assert differ > 0  # the priority search's own choice among ties is exercised


def test_pri_search_orbit_tileset(gpu, oracle):
    """PsyV rows of a tileset in its 4 orientations (symmetric tiles give identical rows), frame-tile queries"""
    rng = np.random.default_rng(43)
    P, T = 8, 1500
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = gpu.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                          flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    picks = rows[rng.choice(rows.shape[0], 48, replace=False)]
    qs = np.concatenate([picks, picks + rng.standard_normal((48, 192)).astype(np.float32) * 0.01])
    _check(gpu, oracle, rows, qs, 0.0)


def test_pri_search_empty_and_index_order(gpu, oracle):
    from nncheck import INDEX_ORDER
    with gpu.KDTree(np.zeros((0, 8), np.float32)) as kdt:
        i, e = kdt.pri_search_batch(np.zeros((2, 8), np.float32))
        assert list(i) == [-1, -1] and np.all(e == np.finfo(np.float32).max)
    rng = np.random.default_rng(44)
    data = rng.integers(0, 3, (500, 6)).astype(np.float32)
    qs = data[:20] + 0.5
    with gpu.KDTree(data, split=INDEX_ORDER) as kdt:  # no tree: ann_kdtree_search's answer (lowest index)
        gi, ge = kdt.pri_search_batch(qs)
    oi, oe = oracle.nn_batch(data, qs)
    assert np.array_equal(gi, oi) and np.array_equal(ge.view(np.uint32), oe.view(np.uint32))

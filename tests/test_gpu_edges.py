"""Edge cases of the drop-in surface on the GPU, each against the oracle: zero queries, a single
candidate, a single query, query counts that are not multiples of the 32-query MFMA blocks, k larger than
the dataset, orbit datasets with a lone (symmetric) tile, NaN-free extreme-but-finite descriptors, and
an empty frame through tiler_frame_tiling."""
import numpy as np
import pytest
from nncheck import INDEX_ORDER, check_nn

from tiler_amd import synth

pytestmark = pytest.mark.gpu


def test_zero_queries(gpu):
    data = np.random.default_rng(1).normal(0, 1, (100, 192)).astype(np.float32)
    with gpu.KDTree(data) as kdt:
        i, e = kdt.search_batch(np.zeros((0, 192), np.float32))
        assert i.size == 0 and e.size == 0


def test_single_candidate_and_single_query(gpu, oracle):
    rng = np.random.default_rng(2)
    data = rng.normal(0, 1, (1, 192)).astype(np.float32)
    q = rng.normal(0, 1, (5, 192)).astype(np.float32)
    with gpu.KDTree(data) as kdt:
        i1, e1 = kdt.search(q[0])
    oi, oe = oracle.nn_batch(data, q)
    check_nn(gpu, oracle, data, q)
    assert i1 == 0 and np.float32(e1) == oe[0]


@pytest.mark.parametrize("nq", [1, 31, 33, 65, 511, 513])
def test_ragged_query_counts_orbit(gpu, oracle, nq):
    """Orbit path with query counts around the 32-query block and 512-query workgroup edges."""
    rng = np.random.default_rng(nq)
    tiles, thm, tvm = synth.tileset(rng, 300)
    pals = synth.palettes(rng, 4)
    used = synth.used_one_palette(rng.integers(0, 4, 300).astype(np.int32), 4)
    ods, *_ = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    q = oracle.psyv_batch(nq, rgb=synth.frame_tiles(rng, nq), flags=2).astype(np.float32)
    st = check_nn(gpu, oracle, ods, q)
    assert st["orbit_search"] == 1


def test_k_larger_than_dataset(gpu, oracle):
    rng = np.random.default_rng(4)
    data = rng.integers(0, 16, (5, 64)).astype(np.float32)
    q = rng.integers(0, 16, (3, 64)).astype(np.float32)
    check_nn(gpu, oracle, data, q, k=8)
    with gpu.KDTree(data) as kdt:
        gi, ge = kdt.search_batch(q, k=8)
    assert (gi[:, 5:] == -1).all()


def test_lone_symmetric_tile_orbit(gpu, oracle):
    """A dataset of one fully symmetric tile in 4 orientations (4 identical rows) and one plain tile:
    every query's winner is the first-found (kd order) / lowest index (index order) among equal rows."""
    t = np.zeros((2, 64), np.uint8)
    t[0] = 5
    t[1] = np.arange(64) % 16
    thm = np.zeros(2, np.uint8)
    tvm = np.zeros(2, np.uint8)
    pals = synth.palettes(np.random.default_rng(5), 1)
    used = np.ones((1, 2, 4), np.uint8)
    ods, *_ = oracle.build_ft_dataset(used, t, thm, tvm, pals)
    rng = np.random.default_rng(6)
    q = np.concatenate([ods, oracle.psyv_batch(40, rgb=synth.frame_tiles(rng, 40), flags=2)]).astype(np.float32)
    check_nn(gpu, oracle, ods, q)
    with gpu.KDTree(ods, split=INDEX_ORDER) as kdt:
        gi, _ = kdt.search_batch(q)
    assert gi[1] == 0 and gi[3] == 0  # index order: the symmetric tile's mirrors resolve to its first row


def test_empty_frame_through_frame_tiling(gpu):
    from tiler_amd.frame_tiling import KeyframeTiler
    wl = synth.make_workload(7, 64, 64, 1, 64, n_palettes=4)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    t, p, h, v, e = kt.do_frame_tiling(np.zeros((0, 64), np.int32))
    assert t.size == 0 and e.size == 0
    kt.finish_frame_tiling()


def test_tiler_init_refuses_rebinding(gpu):
    """Once bound (explicitly or implicitly), the library stays on its device: tiler_init on another device
    fails loudly instead of silently running later calls on the first one (one process per GPU)."""
    lib = gpu.load()
    assert lib.tiler_init(0) == 0
    assert lib.tiler_init(1) == -1
    assert "already bound to device 0" in gpu.last_error()


def test_nonfinite_dataset_builds_and_searches(gpu):
    """a dataset with NaN keys on the root's cut dimension, large enough (> 1,024 rows per node) for the
    workgroup-parallel annMedianSplit (kd_median_big_kernel), NaN pivots included.  The build must stay inside the
    node (NaN is a stopper for both Hoare scans) and leave a permutation; the search runs the exhaustive tier.  What
    ANN returns on NaN distances is order-dependent (a NaN key in ANNmin_k is never displaced), so only sanity is
    asserted for the result: each answer is a real row at its own distance, and no finite row is closer than a finite
    answer would make it... which ANN itself does not promise once a NaN key sits in its list (r04a: 1 of 64 queries
    returned a finite row above the finite minimum, as a NaN-stuck ANNmin_k would), so that part is not asserted."""
    rng = np.random.default_rng(33)
    n, d = 5000, 192
    data = rng.normal(0, 1, (n, d)).astype(np.float32)
    data[:, 0] = rng.integers(0, 1000, n).astype(np.float32)  # the widest spread: the root cuts dimension 0
    data[rng.random(n) < 0.15, 0] = np.nan
    data[rng.random(n) < 0.02, 5] = np.inf
    data[n // 2, 0] = np.nan  # the first pivot of the root's quickselect
    q = rng.normal(0, 1, (96, d)).astype(np.float32)  # > 64: the MFMA path (not the small-batch scan)
    q[:, 0] = rng.integers(0, 1000, 96).astype(np.float32)
    with gpu.KDTree(data) as kdt:
        pos = kdt.positions()
        gi, ge = kdt.search_batch(q)
        st = kdt.stats()
    assert sorted(pos.tolist()) == list(range(n))  # a permutation: nothing written outside the nodes
    with np.errstate(invalid="ignore", over="ignore"):
        dist = np.zeros((q.shape[0], n), np.float32)
        for j in range(d):  # the reference's sequential fp32 sum, dimension order
            t = q[:, j:j + 1] - data[None, :, j]
            dist = dist + t * t
    best = np.array([np.min(r[~np.isnan(r)]) for r in dist], np.float32)
    assert st["exhaustive_queries"] == q.shape[0]
    assert ((gi >= 0) & (gi < n)).all()
    assert np.array_equal(dist[np.arange(q.shape[0]), gi].view(np.uint32), ge.view(np.uint32))
    assert np.all(np.isnan(ge) | (ge >= best))


def test_tier2_overflow_on_fresh_index_exact(gpu, oracle):
    """a fresh index sizes its generic tier-2 slots from the recent count of OTHER indexes.  Here an
    index whose searches need no tier 2 runs first, then a fresh index where every one of 70,000 queries ties 16
    identical copies (its lane lists fill with equal keys: all go to tier 2, more than the 65,536 slots of one
    chunk).  Whatever the slots, every answer must be exact (the overflow goes to the exhaustive tier 3): a sample of
    3,000 queries equals the restated lowest-index scan."""
    rng = np.random.default_rng(71)
    plain = rng.normal(0, 1, (20000, 192)).astype(np.float32)
    with gpu.KDTree(plain, split=INDEX_ORDER) as kdt:
        kdt.search_batch(plain[:4096] + 0.5)
        assert kdt.stats()["fallback_queries"] < 1000
    base = rng.normal(0, 1, (2048, 192)).astype(np.float32)
    data = np.tile(base, (16, 1))
    pick = rng.integers(0, 2048, 70000)
    q = base[pick] + rng.normal(0, 1e-3, (70000, 192)).astype(np.float32)
    with gpu.KDTree(data, split=INDEX_ORDER) as kdt:
        gi, ge = kdt.search_batch(q)
        st = kdt.stats()
    assert st["orbit_search"] == 0 and st["fallback_queries"] + st["exhaustive_queries"] > 65536, st
    s = np.random.default_rng(5).choice(q.shape[0], 3000, replace=False)
    oi, oe = oracle.nn_batch(data, q[s])
    assert np.array_equal(gi[s], oi)
    assert np.array_equal(ge[s].view(np.uint32), oe.view(np.uint32))
    assert (gi < 2048).all()  # the lowest-index copy


def test_forced_replay_exact(gpu, oracle):
    """tiler_debug_force_replay: ANN's pruning check vouches for nothing, so every kd-order query -- the coalesced
    small-batch path (scan, merge + check, replay) and the MFMA path (verify kernel, replay) -- runs the exact
    annkSearch replay; every answer must still equal the restated search, k = 1 and k = 8."""
    lib = gpu.load()
    rng = np.random.default_rng(81)
    tiles, thm, tvm = synth.tileset(rng, 400)
    pals = synth.palettes(rng, 4)
    used = synth.used_one_palette(rng.integers(0, 4, 400).astype(np.int32), 4)
    ods, *_ = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    q = oracle.psyv_batch(300, rgb=synth.frame_tiles(rng, 300), flags=2).astype(np.float32)
    gen = rng.normal(0, 1, (3000, 192)).astype(np.float32)
    gq = gen[rng.integers(0, 3000, 200)] + rng.normal(0, 0.05, (200, 192)).astype(np.float32)
    ints = rng.integers(0, 16, (2000, 64)).astype(np.float32)
    iq = ints[rng.integers(0, 2000, 100)]
    assert lib.tiler_debug_force_replay(1) == 0
    try:
        for nq in (5, 300):  # the scan path (<= 64 queries) and the MFMA path
            check_nn(gpu, oracle, ods, q[:nq])
        st = check_nn(gpu, oracle, gen, gq)
        assert st["kd_replayed"] == gq.shape[0], st
        check_nn(gpu, oracle, ints, iq[:10], k=8)
        st8 = check_nn(gpu, oracle, ints, iq, k=8)
        assert st8["kd_replayed"] > 0, st8
    finally:
        lib.tiler_debug_force_replay(0)

"""Exact ties inside every per-lane / per-thread candidate list of the search.

Until round 5 the small-batch merge folded up to 16 splits per lane into a per-lane K-list with a shifting insertion
whose tie test calls the kd-tree walk; this toolchain miscompiled that loop (the lanes whose tie test succeeds at the
last step lose list[0] and hold list[1] twice: kdorder_dev.hpp kd_list_insert, tools/merge_tie_repro.hip, DESIGN §4
"A k = 8 correctness fix").  The merge is now wide (one split per thread, no per-lane list) and every remaining
per-thread list with tie-order insertions (scan, tier 2, tier 3) uses the two-phase kd_list_insert.  Each test below
puts identical rows where one list holds several of them and compares the k results with the restated ANN search
(oracle/ann_kdtree.c) and the lowest-index scan, bit for bit (nncheck: small batches both through the exhaustive scan
and, with it disabled, through the MFMA shortlist and its tiers):

* the merge: one copy at the head of splits 11, 75, 139, 203, 523 and 843 of a 262,144-row plain index (1,024 splits
  of 256 rows): all six were lane 11's in the removed one-wave merge -- the C3 failure's layout (profiles/r05k8);
* the scan's per-thread lists: a 1,048,576-row index (1,024 rows per split, 4 rows per thread), 4 copies in one
  thread of one split and 4 more in the same thread of another split;
* the generic shortlist's per-lane lists and tier 2's per-lane lists: 600 scattered copies in a 40,000-row index (every
  shortlist lane list overflows below the threshold -> tier 2 with several copies per lane), 2,500 (-> tier 3);
* the mirror-orbit shortlist and scan: a tileset where one flat tile occurs 160 times and one H-symmetric tile 160
  times in one palette (640 + 320 identical rows in 320 orbit groups).
"""
import numpy as np
import pytest

from nncheck import check_nn

pytestmark = pytest.mark.gpu


def _copies_at(rows, q, at):
    rows = rows.copy()
    rows[np.asarray(at)] = q
    return rows


@pytest.mark.parametrize("k", [1, 8])
def test_merge_ties_across_one_lanes_splits(gpu, oracle, k):
    rng = np.random.default_rng(600 + k)
    n, d, split = 262144, 64, 256
    rows = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    at = [sp * split + int(rng.integers(0, split)) for sp in (11, 75, 139, 203, 523, 843)]
    rows = _copies_at(rows, q, at)
    qs = np.stack([q, rows[5] + np.float32(0.01), q + np.float32(1e-3)])
    for nq in (1, 3):
        check_nn(gpu, oracle, rows, qs[:nq], k=k)


@pytest.mark.parametrize("k", [1, 8])
def test_scan_thread_list_ties(gpu, oracle, k):
    rng = np.random.default_rng(610 + k)
    n, d, split = 1 << 20, 8, 1024
    rows = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    t = int(rng.integers(0, 256))
    at = [sp * split + t + 256 * m for sp in (40, 104) for m in range(4)]  # one thread, two splits, 4 rounds each
    rows = _copies_at(rows, q, at)
    qs = np.stack([q, q + np.float32(1e-3), rows[77]])
    for nq in (1, 3):
        check_nn(gpu, oracle, rows, qs[:nq], k=k)


@pytest.mark.parametrize("k", [1, 8])
@pytest.mark.parametrize("copies", [600, 2500])
def test_shortlist_and_tier_list_ties(gpu, oracle, k, copies):
    rng = np.random.default_rng(620 + copies + k)
    n, d = 40000, 192
    rows = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal(d).astype(np.float32)
    rows = _copies_at(rows, q, rng.choice(n, copies, replace=False))
    picks = rows[rng.choice(n, 70, replace=False)]
    qs = np.concatenate([q[None], q[None] + np.float32(1e-3), picks]).astype(np.float32)
    st = check_nn(gpu, oracle, rows, qs[:2], k=k)  # small batch: the scan, then the MFMA tiers
    assert st["fallback_queries"] + st["exhaustive_queries"] >= 1
    check_nn(gpu, oracle, rows, qs, k=k)  # 72 queries: the MFMA path only


@pytest.mark.parametrize("k", [1, 8])
def test_orbit_list_ties(gpu, oracle, k):
    from tiler_amd import synth
    rng = np.random.default_rng(640 + k)
    P, T = 2, 3000
    pals = synth.palettes(rng, P)
    raw = rng.integers(0, 16, (T, 8, 8)).astype(np.uint8)
    raw[:160] = 3                                           # one flat tile, 160 times: 4 identical mirrors each
    sym = rng.integers(0, 16, (8, 8)).astype(np.uint8)
    sym[:, 4:] = sym[:, 3::-1]
    raw[160:320] = sym                                      # one H-symmetric tile, 160 times: 2 distinct rows each
    tiles, thm, tvm = synth.prepare_tile_mirrors(raw.reshape(T, 64))
    tile_pal = rng.integers(0, P, T).astype(np.int32)
    tile_pal[:320] = 0
    ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
    rows = gpu.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                          flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    with gpu.KDTree(rows) as kdt:
        assert kdt.stats()["orbit_groups"] > 0
    flat = rows[np.nonzero(ds.tile_of == 0)[0][0]]
    symr = rows[np.nonzero(ds.tile_of == 160)[0]]
    others = rows[rng.choice(rows.shape[0], 70, replace=False)]
    qs = np.concatenate([flat[None], symr[:2], flat[None] + np.float32(1e-3), others]).astype(np.float32)
    check_nn(gpu, oracle, rows, qs[:4], k=k)  # the orbit scan, then the orbit shortlist
    check_nn(gpu, oracle, rows, qs, k=k)      # 74 queries: the orbit shortlist only

"""GPU parity of the mirror-orbit search path (tiler_amd/csrc/orbit.hip) against the CPU restatement.

The orbit path scores the 4 H/V mirrors of a tile (PrepareFrameTiling.DoPsyV emission order,
main.pas:3883-3919) with one MFMA pass; results must stay bit-identical to the exhaustive reference-order
scan: index, fp32 distance, and on exact ties ANN's kd-tree first-found candidate
(default) or the lowest index (split = TILER_SPLIT_INDEX_ORDER) -- nncheck.check_nn runs both.
"""
import numpy as np
import pytest
from nncheck import INDEX_ORDER, check_nn

from tiler_amd import synth

pytestmark = pytest.mark.gpu


def _ft_rows(oracle, seed, T, P, used_fn=None):
    rng = np.random.default_rng(seed)
    tiles, thm, tvm = synth.tileset(rng, T)
    pals = synth.palettes(rng, P)
    if used_fn is None:
        used = synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P)
    else:
        used = used_fn(rng, P, T)
    ods, ot, op, oa = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    return rng, ods, ot, op, oa


def _check(gpu, oracle, data, qs, expect_orbit=True):
    st = check_nn(gpu, oracle, data, qs)
    if expect_orbit:
        assert st["orbit_search"] == 1 and st["orbit_groups"] > 0, st
    return st


def test_orbit_full_mirror_sets(gpu, oracle):
    """P_eff = 1: every tile in 4 orientations (the benchmark's dataset shape), frame-tile queries."""
    rng, ods, *_ = _ft_rows(oracle, 31, 3000, 16)
    q = oracle.psyv_batch(2500, rgb=synth.frame_tiles(rng, 2500), flags=2).astype(np.float32)
    st = _check(gpu, oracle, ods, q)
    assert st["orbit_groups"] == ods.shape[0] // 4


def test_orbit_partial_mirror_sets(gpu, oracle):
    """Medium-quality style used tables: random subsets of (palette, tile, orientation), so orbits have holes
    and groups start at any orientation."""
    def used_fn(rng, P, T):
        u = (rng.random((P, T, 4)) < 0.3).astype(np.uint8)
        return u
    rng, ods, *_ = _ft_rows(oracle, 32, 900, 6, used_fn)
    q = oracle.psyv_batch(1500, rgb=synth.frame_tiles(rng, 1500), flags=2).astype(np.float32)
    _check(gpu, oracle, ods, q)


def test_orbit_exact_matches_and_mirror_ties(gpu, oracle):
    """Queries that ARE candidates (distance 0): symmetric tiles tie across mirrors."""
    rng, ods, *_ = _ft_rows(oracle, 33, 1200, 8)
    pick = rng.integers(0, ods.shape[0], 700)
    q = ods[pick].copy()
    st = _check(gpu, oracle, ods, q)
    assert st["exhaustive_queries"] == 0


def test_orbit_duplicate_tiles_force_overflow(gpu, oracle):
    """Many identical tiles (same palette) make equal-distance groups larger than the shortlists: the
    overflow tiers must still return the right winner under both tie rules."""
    rng = np.random.default_rng(34)
    tiles, thm, tvm = synth.tileset(rng, 400)
    tiles[200:] = tiles[0]
    thm[200:] = thm[0]
    tvm[200:] = tvm[0]
    pals = synth.palettes(rng, 2)
    used = np.zeros((2, 400, 4), np.uint8)
    used[0] = 1
    ods, *_ = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    q = np.concatenate([ods[:8], oracle.psyv_batch(300, rgb=synth.frame_tiles(rng, 300), flags=2)]).astype(np.float32)
    st = _check(gpu, oracle, ods, q)
    assert st["fallback_queries"] + st["exhaustive_queries"] > 0


def test_orbit_large_values_scaled(gpu, oracle):
    """Descriptors scaled far beyond fp16 range (power-of-two dataset scale) and tiny ones."""
    rng, ods, *_ = _ft_rows(oracle, 35, 800, 4)
    q = oracle.psyv_batch(600, rgb=synth.frame_tiles(rng, 600), flags=2).astype(np.float32)
    for s in (1e6, 1e-6):
        _check(gpu, oracle, (ods * np.float32(s)).astype(np.float32), (q * np.float32(s)).astype(np.float32))


def test_orbit_not_used_for_unstructured_data(gpu, oracle):
    rng = np.random.default_rng(36)
    data = rng.normal(0, 1, (3000, 192)).astype(np.float32)
    q = rng.normal(0, 1, (500, 192)).astype(np.float32)
    st = _check(gpu, oracle, data, q, expect_orbit=False)
    assert st["orbit_groups"] == 0 and st["orbit_search"] == 0


def test_orbit_c2_frame_sampled(gpu, oracle):
    """C2 shape (720p frame, 16k tileset x 4 mirrors = 65,536 candidates): the whole frame through
    tiler_frame_tiling, a bounded sample checked against the exhaustive oracle scan."""
    from tiler_amd.frame_tiling import KeyframeTiler
    wl = synth.make_workload(41, 1280, 720, 1, 16384, n_palettes=128)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    g = kt.do_frame_tiling(wl.frame_rgb[0])
    st = kt.kdt.stats()
    used = synth.used_one_palette(wl.tile_pal, 128)
    ods, ot, op, oa = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    pick = np.random.default_rng(1).choice(wl.tiles_per_frame, 500, replace=False)
    o = oracle.frame_tiling(wl.frame_rgb[0][pick], ods, ot, op, oa)
    for a, b in zip(g[:4], o[:4]):
        assert np.array_equal(np.asarray(a)[pick], b)
    assert np.array_equal(np.asarray(g[4])[pick].view(np.uint32), o[4].view(np.uint32))
    kt.finish_frame_tiling()
    assert st["orbit_search"] == 1


def test_orbit_c3_self_queries(gpu, oracle):
    """Full C3 candidate set (64k tileset x 4 mirrors = 262,144 rows, built on the GPU): querying rows of
    the dataset must return distance 0 and, under index order, the LOWEST index holding an identical row
    (size-independent property of the exact search, covers symmetric tiles whose mirrors coincide); under
    ANN's order the very candidate oracle/ann_kdtree.c finds first."""
    rng = np.random.default_rng(43)
    P, T = 128, 65536
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = gpu.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                          flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    pick = rng.choice(rows.shape[0], 3000, replace=False)
    with gpu.KDTree(rows, split=INDEX_ORDER) as kdt:
        gi, ge = kdt.search_batch(rows[pick])
        st = kdt.stats()
    assert st["orbit_search"] == 1 and st["orbit_groups"] == T
    assert (ge == 0).all()
    # lowest index with an identical row
    v = np.ascontiguousarray(rows).view(np.dtype((np.void, rows.shape[1] * 4))).ravel()
    _, first = np.unique(v, return_index=True)
    inv = np.unique(v, return_inverse=True)[1].ravel()
    assert np.array_equal(gi, first[inv[pick]])
    # ANN's order: the kd-tree's first-found copy
    with gpu.KDTree(rows) as kdt:
        ki, ke = kdt.search_batch(rows[pick])
        pos = kdt.positions()
    okd = oracle.KDTree(rows)
    assert np.array_equal(pos, okd.positions()), "kd-tree leaf order differs from ANN's"
    oi, oe = okd.search_batch(rows[pick])
    okd.close()
    assert (ke == 0).all() and np.array_equal(ki, oi)
    assert np.array_equal(rows[ki].view(np.uint32), rows[pick].view(np.uint32))


def test_ann_tie_order_c3_frame_queries(gpu, oracle):
    """SURVEY.md 8(a) a8 at the headline size: a C3 keyframe dataset (64k tileset x 4 mirrors, 20 % symmetric
    tiles) and 3,072 frame-tile queries (smooth / textured / flat mix) through
    tiler_frame_tiling; tile, palette and mirror flags must equal ANN 1.1.2's kd-tree search (oracle)."""
    from tiler_amd.frame_tiling import KeyframeTiler
    wl = synth.make_workload(45, 1920, 1080, 1, 65536, n_palettes=128)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    q = wl.frame_rgb[0][:3072]
    g = kt.do_frame_tiling(q)
    st = kt.kdt.stats()
    kt.finish_frame_tiling()
    used = synth.used_one_palette(wl.tile_pal, 128)
    ods, ot, op, oa = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    o = oracle.frame_tiling(q, ods, ot, op, oa)
    assert np.array_equal(np.asarray(g[4]).view(np.uint32), o[4].view(np.uint32))
    for a, b in zip(g[:4], o[:4]):
        assert np.array_equal(a, b), f"{np.count_nonzero(a != b)} of {q.shape[0]} items differ"
    # the tie rule matters here: lowest-index resolution differs from ANN's on many of these queries
    oi = oracle.frame_tiling(q, ods, ot, op, oa, kd_order=False)
    n_tie = int(np.count_nonzero((oi[0] != o[0]) | (oi[2] != o[2]) | (oi[3] != o[3])))
    assert n_tie > 0
    assert st["orbit_search"] == 1 and st["tie_order"] == 0


def test_c5_frame_queries_vs_ann(gpu, oracle):
    """BASELINE C5 candidate set at full size: a 256k tileset x 4 mirrors = 1,048,576 candidates (805 MB of fp32
    rows in HBM), 1,024 4K frame-tile queries through tiler_frame_tiling against ANN's kd-tree search on the
    host (oracle/ann_kdtree.c, 16 threads): tile, palette, mirror flags and distance bit for bit."""
    from tiler_amd.frame_tiling import KeyframeTiler
    rng = np.random.default_rng(55)
    P, T = 128, 262144
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    tile_pal = rng.integers(0, P, T).astype(np.int32)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
    assert ds.tile_of.size == 4 * T
    q = synth.frame_tiles(rng, 1024)  # the 4K frame-tile mix (smooth / textured / flat)
    kt = KeyframeTiler(tiles, thm, tvm, pals, ds)
    g = kt.do_frame_tiling(q)
    st = kt.kdt.stats()
    rows = kt.rows
    kt.finish_frame_tiling()
    assert st["orbit_search"] == 1 and st["tie_order"] == 0 and st["orbit_groups"] == T
    o = oracle.frame_tiling(q, rows, ds.tile_of, ds.pal_of, ds.attrs)
    assert np.array_equal(np.asarray(g[4]).view(np.uint32), o[4].view(np.uint32))
    for a, b in zip(g[:4], o[:4]):
        assert np.array_equal(a, b), f"{np.count_nonzero(a != b)} of {q.shape[0]} items differ"

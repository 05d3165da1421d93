"""GPU parity: libANN.so (HIP, gfx950) against the CPU restatement (oracle/) on seeded inputs.

Bar: descriptors fp64 bit-exact; distances fp32 bit-exact; tile / palette / mirror
indices bit-exact under ANN's kd-tree tie order (the reference's, default) and under the lowest-index
opt-in (split = TILER_SPLIT_INDEX_ORDER).
"""
import numpy as np
import pytest
from nncheck import INDEX_ORDER, check_nn

from tiler_amd import synth

pytestmark = pytest.mark.gpu

PSYV_FLAG_SETS = [2, 0, 8, 2 | 16, 2 | 32, 2 | 48, 8 | 16 | 32, 1 | 2, 1 | 8, 1 | 2 | 16 | 32, 1 | 8 | 48]


def _rgb_tiles(rng, n):
    t = synth.frame_tiles(rng, n)
    # extremes: black, white, pure primaries, single-pixel impulses
    t[:6] = np.array([0, 0xFFFFFF, 0xFF, 0xFF00, 0xFF0000, 0x808080], np.int32)[:, None]
    t[6, 17] = 0xFFFFFF
    return t


@pytest.mark.parametrize("gamma", [-1, 0, 1])
def test_psyv_rgb_bit_exact(gpu, oracle, gamma):
    rng = np.random.default_rng(100 + gamma)
    n = 600
    rgb = _rgb_tiles(rng, n)
    for flags in [f for f in PSYV_FLAG_SETS if not f & 1]:
        g64, g32 = gpu.psyv_batch(rgb=rgb, flags=flags, gamma=gamma, want64=True, want32=True)
        o64 = oracle.psyv_batch(n, rgb=rgb, flags=flags, gamma=gamma)
        assert np.array_equal(g64.view(np.uint64), o64.view(np.uint64)), f"flags={flags}"
        assert np.array_equal(g32.view(np.uint32), o64.astype(np.float32).view(np.uint32))


def test_psyv_palette_bit_exact(gpu, oracle):
    rng = np.random.default_rng(7)
    T, P, n = 300, 9, 900
    pp = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    pals = synth.palettes(rng, P)
    tile_of = rng.integers(0, T, n).astype(np.int32)
    pal_of = rng.integers(0, P, n).astype(np.int32)
    fper = (rng.integers(0, 4, n) * 16).astype(np.uint8)
    for flags in (1 | 2, 1 | 8, 1):
        g64, _ = gpu.psyv_batch(palpix=pp, tile_of=tile_of, palettes=pals, pal_of=pal_of, flags_per=fper,
                                flags=flags, gamma=-1)
        o64 = oracle.psyv_batch(n, palpix=pp[tile_of], pals=pals, pal_of=pal_of, flags_per=fper, flags=flags)
        assert np.array_equal(g64.view(np.uint64), o64.view(np.uint64)), f"flags={flags}"


def _check_nn(gpu, oracle, data, qs):
    return check_nn(gpu, oracle, data, qs)


def test_nn_random_descriptors(gpu, oracle):
    rng = np.random.default_rng(1)
    wl = synth.make_workload(11, 160, 80, 2, 2000, n_palettes=8)
    _, data = gpu.psyv_batch(palpix=wl.tiles, tile_of=wl.ds.tile_of, palettes=wl.palettes, pal_of=wl.ds.pal_of,
                             flags_per=wl.ds.psyv_flags, flags=3, want64=False, want32=True)
    _, qs = gpu.psyv_batch(rgb=wl.frame_rgb.reshape(-1, 64), flags=2, want64=False, want32=True)
    st = _check_nn(gpu, oracle, data, qs)
    assert st["queries"] == qs.shape[0]
    # near-duplicate queries: a candidate row itself plus tiny perturbations (tight shortlists)
    q2 = data[rng.integers(0, data.shape[0], 300)].copy()
    q2[100:] += rng.normal(0, 1e-4, q2[100:].shape).astype(np.float32)
    _check_nn(gpu, oracle, data, q2)


def test_nn_ties_both_orders(gpu, oracle):
    rng = np.random.default_rng(2)
    base = rng.normal(0, 1, (500, 192)).astype(np.float32)
    data = np.concatenate([base, base[::-1], base[:50]])  # every row duplicated, some three times
    qs = np.concatenate([base[:100], rng.normal(0, 1, (100, 192)).astype(np.float32)])
    _check_nn(gpu, oracle, data, qs)


def test_nn_overflow_fallback(gpu, oracle):
    # 300 identical candidates: every lane list overflows below the threshold -> exact rescan path
    rng = np.random.default_rng(3)
    data = np.repeat(rng.normal(0, 1, (1, 192)).astype(np.float32), 300, 0)
    data = np.concatenate([rng.normal(0, 1, (700, 192)).astype(np.float32), data])
    qs = data[[0, 5, 700, 950]] + np.float32(1e-3)
    st = _check_nn(gpu, oracle, data, qs)
    assert st["fallback_queries"] >= 1  # tier 2 (MFMA collect + exact rescoring)
    # 1500 identical candidates overflow the tier-2 buffer too -> tier 3 exhaustive scan
    many = np.repeat(data[700:701], 1500, 0)
    data3 = np.concatenate([data[:700], many])
    st3 = _check_nn(gpu, oracle, data3, data3[[3, 800]] + np.float32(1e-3))
    assert st3["exhaustive_queries"] >= 1


def test_nn_generic_dims(gpu, oracle):
    rng = np.random.default_rng(4)
    for d in (3, 17, 64, 100, 256, 300):
        data = rng.normal(0, 3, (3000, d)).astype(np.float32)
        qs = rng.normal(0, 3, (257, d)).astype(np.float32)
        _check_nn(gpu, oracle, data, qs)


def test_knn_palette_index_preselection(gpu, oracle):
    """k=8 on 64-d palette-index rows (PrepareGlobalFT dataset, main.pas:3779/3830): exact integer keys."""
    rng = np.random.default_rng(5)
    tiles, _, _ = synth.tileset(rng, 1500)
    gds, gt, ga = oracle.prepare_global_ds(tiles)
    qs = tiles[rng.integers(0, 1500, 400)].astype(np.float32)
    qs[200:] = rng.integers(0, 16, (200, 64))
    with gpu.KDTree(gds) as kdt:
        assert kdt.stats()["exact_integer"] == 1
    check_nn(gpu, oracle, gds, qs, k=8)


def test_knn_heavy_ties(gpu, oracle):
    """k=8 where dozens of candidates share the k-th distance (2-colour tiles): a lane list full of equal keys may
    hide the one ANN finds first, so the tier-1 overflow check must hold for exact integer keys too."""
    rng = np.random.default_rng(15)
    tiles = (rng.random((2000, 64)) < 0.1).astype(np.uint8)
    gds, gt, ga = oracle.prepare_global_ds(tiles)
    qs = np.concatenate([tiles[rng.integers(0, 2000, 200)], (rng.random((200, 64)) < 0.1)]).astype(np.float32)
    st = check_nn(gpu, oracle, gds, qs, k=8)
    assert st["fallback_queries"] > 0
    check_nn(gpu, oracle, gds, qs, k=1)


def test_reference_call_shapes(gpu, oracle):
    """ann_kdtree_search / search_multi one query at a time, as main.pas:4027 and 3830 call them."""
    rng = np.random.default_rng(6)
    data = rng.normal(0, 1, (4000, 192)).astype(np.float32)
    data[7] = data[3]  # an exact duplicate: a tie for queries near it
    okd = oracle.KDTree(data)
    for split in (0, INDEX_ORDER):
        with gpu.KDTree(data, split=split) as kdt:
            for j in range(6):
                q = rng.normal(0, 1, 192).astype(np.float32) if j < 5 else data[3] + np.float32(1e-4)
                i, e = kdt.search(q)
                if split == 0:
                    oi, oe = okd.search_batch(q[None])
                    oi, oe = int(oi[0]), float(oe[0])
                else:
                    oi, oe = oracle.nn(data, q)
                assert (i, np.float32(e)) == (oi, np.float32(oe)), (split, j)
                for k in (1, 8, 20):
                    ii, ee = kdt.search_multi(q, k)
                    if split == 0:
                        oi2, oe2 = okd.search_batch(q[None], k=k)
                        oi2, oe2 = oi2.reshape(-1), oe2.reshape(-1)
                    else:
                        oi2, oe2 = oracle.knn(data, q, k)
                    assert np.array_equal(ii, oi2) and np.array_equal(ee, oe2), (split, j, k)
    okd.close()
    with gpu.KDTree(np.zeros((0, 192), np.float32)) as empty:
        idx, err = empty.search_batch(np.zeros((2, 192), np.float32))
        assert (idx == -1).all()


def test_frame_tiling_end_to_end_c1(gpu, oracle):
    """C1 shape (320x240, 8x8) with a 1k tileset: DoFrameTiling tilemap items bit-exact."""
    from tiler_amd.frame_tiling import KeyframeTiler
    wl = synth.make_workload(21, 320, 240, 3, 1000, n_palettes=16)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    used = synth.used_one_palette(wl.tile_pal, 16)
    ods, otile, opal, oattr = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    assert np.array_equal(kt.rows.view(np.uint32), ods.view(np.uint32))
    assert np.array_equal(otile, wl.ds.tile_of) and np.array_equal(opal, wl.ds.pal_of)
    assert np.array_equal(oattr, wl.ds.attrs)
    for f in range(wl.frames):
        g = kt.do_frame_tiling(wl.frame_rgb[f])
        o = oracle.frame_tiling(wl.frame_rgb[f], ods, otile, opal, oattr)
        for a, b in zip(g[:4], o[:4]):
            assert np.array_equal(a, b)
        assert np.array_equal(g[4].view(np.uint32), o[4].view(np.uint32))
    kt.finish_frame_tiling()


def test_frame_tiling_small_batches_on_orbit_index(gpu, oracle):
    """DoFrameTiling batches of <= 64 tiles on a mirror-orbit index (20 % symmetric tiles, so equal
    distances among a tile's mirrors) take the small-batch exact scan by default; with the scan disabled
    (tiler_set_scan_limits(0, 0)) they take the orbit MFMA tiers.  Both must give the restatement's tilemap items,
    mirror flags and errors bit for bit."""
    from tiler_amd.frame_tiling import KeyframeTiler
    wl = synth.make_workload(29, 320, 240, 1, 3000, n_palettes=16)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    assert kt.kdt.stats()["orbit_groups"] > 0
    used = synth.used_one_palette(wl.tile_pal, 16)
    ods, otile, opal, oattr = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    lib = gpu.load()
    try:
        for limits in ((64, 16), (0, 0)):
            assert lib.tiler_set_scan_limits(*limits) == 0
            for q0, nq in ((0, 1), (5, 17), (100, 64)):
                rgb = wl.frame_rgb[0][q0:q0 + nq]
                g = kt.do_frame_tiling(rgb)
                o = oracle.frame_tiling(rgb, ods, otile, opal, oattr)
                for a, b in zip(g[:4], o[:4]):
                    assert np.array_equal(a, b), (limits, q0, nq)
                assert np.array_equal(g[4].view(np.uint32), o[4].view(np.uint32)), (limits, q0, nq)
    finally:
        lib.tiler_set_scan_limits(64, 16)
    kt.finish_frame_tiling()


def test_frame_tiling_flat_tiles_last_matches_small_batches(gpu):
    """A batch of >= 8192 tiles runs with its flat tiles moved last (their shortlist workgroups compute isotypic block
    0 only, nn_frame_tiling_dev / orbit_search); per-frame batches below that size keep the tile order.  Both must
    give the same tilemap items and errors bit for bit (the per-frame path is checked against the oracle above)."""
    from tiler_amd.frame_tiling import KeyframeTiler
    # >= 1,024 blocks of 32 mirror groups: the grouping is enabled from that shortlist length (nn_frame_tiling_dev)
    wl = synth.make_workload(23, 320, 240, 8, 40000, n_palettes=16)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    assert kt.kdt.stats()["orbit_groups"] >= 1024 * 32
    frames = np.stack([wl.frame_rgb[f] for f in range(wl.frames)])
    Q = frames.shape[1]
    flat = (frames.reshape(-1, 64) == frames.reshape(-1, 64)[:, :1]).all(axis=1)
    assert frames.shape[0] * Q >= 8192 and 0 < flat.sum() < flat.size
    big = kt.do_frame_tiling(frames.reshape(-1, 64))
    assert kt.kdt.stats()["flat_queries"] > 0  # the flat tiles' workgroups ran
    for f in range(wl.frames):
        g = kt.do_frame_tiling(frames[f])
        for a, b in zip(g[:4], big[:4]):
            assert np.array_equal(a, b[f * Q:(f + 1) * Q])
        assert np.array_equal(g[4].view(np.uint32), big[4][f * Q:(f + 1) * Q].view(np.uint32))
    kt.finish_frame_tiling()


def test_frame_tiling_flat_tiles_last_generic_path(gpu, oracle):
    """The same grouping on the generic 16x16x32 shortlist (candidate sets without mirror orbits: one orientation per
    (palette, tile), as real PrepareFrameTiling output mostly is): both operands' fragments carry the three PsyV DC
    dimensions in k-step 0 (dc_first_dim), so the flat workgroups contract k-step 0 only.  The >= 8192-tile batch
    must equal per-frame batches (no grouping) and the oracle (restated ANN search) bit for bit."""
    from tiler_amd.frame_tiling import KeyframeTiler
    rng = np.random.default_rng(29)
    P, T = 16, 6000
    tiles, thm, tvm = synth.tileset(rng, T)
    pals = synth.palettes(rng, P)
    used = np.zeros((P, T, 4), np.uint8)
    for _ in range(2):  # two (palette, orientation) cells per tile, never a whole mirror orbit
        used[rng.integers(0, P, T), np.arange(T), rng.integers(0, 4, T)] = 1
    ds = synth.ft_dataset_from_used(used, thm, tvm)
    kt = KeyframeTiler(tiles, thm, tvm, pals, ds)
    frames = synth.keyframe_frames(rng, 8, 1200)
    flat = (frames.reshape(-1, 64) == frames.reshape(-1, 64)[:, :1]).all(axis=1)
    assert frames.shape[0] * 1200 >= 8192 and 0 < flat.sum() < flat.size
    big = kt.do_frame_tiling(frames.reshape(-1, 64))
    st = kt.kdt.stats()
    assert st["orbit_search"] == 0 and st["flat_queries"] > 0
    for f in range(frames.shape[0]):
        g = kt.do_frame_tiling(frames[f])
        for a, b in zip(g[:4], big[:4]):
            assert np.array_equal(a, b[f * 1200:(f + 1) * 1200])
        assert np.array_equal(g[4].view(np.uint32), big[4][f * 1200:(f + 1) * 1200].view(np.uint32))
    kt.finish_frame_tiling()
    ods, ot, op, oa = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    pick = np.concatenate([np.nonzero(flat)[0][:300], np.nonzero(~flat)[0][:300]])
    o = oracle.frame_tiling(frames.reshape(-1, 64)[pick], ods, ot, op, oa)
    for a, b in zip(big[:4], o[:4]):
        assert np.array_equal(a[pick], b)
    assert np.array_equal(big[4][pick].view(np.uint32), o[4].view(np.uint32))


def test_prepare_frame_tiling_used_table(gpu, oracle):
    """UseOne (k=8 preselection + distinct-err walk) for Fast / Medium / Slow, main.pas:3802-3853."""
    from tiler_amd import frame_tiling as ft
    rng = np.random.default_rng(8)
    P, T = 6, 400
    tiles, thm, tvm = synth.tileset(rng, T)
    cent = rng.normal(0, 1, (P, 192))
    cent[3] = cent[2] + 1e-3  # a close palette pair for Medium
    items_t = rng.integers(0, T, 2000).astype(np.int32)
    items_p = rng.integers(0, P, 2000).astype(np.int32)
    gds = ft.prepare_global_ft(tiles)
    ogds, ogt, oga = oracle.prepare_global_ds(tiles)
    assert np.array_equal(gds.tr_tile, ogt) and np.array_equal(gds.tr_attrs, oga)
    corr_o, hi_o = oracle.palette_corr(cent)
    corr_g, hi_g = ft.palette_corr(cent)
    assert np.array_equal(corr_o, corr_g) and hi_o == hi_g
    for q in (ft.FT_FAST, ft.FT_MEDIUM, ft.FT_SLOW):
        ug = ft.mark_used(gds, tiles, items_p, items_t, P, q, corr_g, hi_g)
        uo = oracle.mark_used(ogds, ogt, oga, items_p, items_t, tiles, P, q, corr_o, hi_o)
        assert np.array_equal(ug, uo), q


def test_prepare_frame_tiling_dev_matches_restatement(gpu, oracle):
    """tiler_prepare_frame_tiling_dev (PrepareFrameTiling main.pas:3791-3967 on the device: distinct items by bitmap,
    UseOne's k = 8 preselection, used bitmap, DoPsyV order, descriptors, index) for Fast / Medium / Slow: the
    keyframe dataset has the restatement's size and the FrameTiling items over it equal oracle.frame_tiling over the
    oracle's dataset (used table -> build_ft_dataset), bit for bit, with ANN's tie order.  Items include -1 (none)
    and repeats; the scratch is reused across the three calls."""
    import torch
    from tiler_amd import frame_tiling as ft
    rng = np.random.default_rng(18)
    P, T = 8, 700
    pals = synth.palettes(rng, P)
    pals[1::2] = pals[0::2] ^ rng.integers(0, 2, pals[1::2].shape)  # near-identical pairs: Medium marks both
    tiles, thm, tvm = synth.tileset(rng, T)
    cent = synth.palette_centroids(pals)
    items_t = rng.integers(0, T, 6000).astype(np.int32)
    items_p = rng.integers(0, P, 6000).astype(np.int32)
    items_t[::97] = -1
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(np.ascontiguousarray(a)).to(dev) for k, a in
         (("t", items_t), ("p", items_p), ("tiles", tiles), ("thm", thm), ("tvm", tvm), ("pals", pals))}
    frames = synth.frame_tiles(rng, 1500)
    gds = ft.prepare_global_ft(tiles)
    ogds, ogt, oga = oracle.prepare_global_ds(tiles)
    corr_o, hi_o = oracle.palette_corr(cent)
    near = ft.near_palettes(cent)
    assert near.sum() > P  # some palette pairs are near
    keep = items_t >= 0
    try:
        for q in (ft.FT_FAST, ft.FT_MEDIUM, ft.FT_SLOW):
            kt, info = ft.prepare_frame_tiling_dev(gds, d["t"].data_ptr(), d["p"].data_ptr(), items_t.size,
                                                   d["tiles"].data_ptr(), d["thm"].data_ptr(), d["tvm"].data_ptr(), T,
                                                   d["pals"].data_ptr(), P, q, near)
            torch.cuda.synchronize(dev)
            uo = oracle.mark_used(ogds, ogt, oga, items_p[keep], items_t[keep], tiles, P, q, corr_o, hi_o)
            assert info["items"] == np.unique(items_p[keep].astype(np.int64) * T + items_t[keep]).size, q
            assert info["candidates"] == int(uo.sum()), q
            ods, ot, op, oa = oracle.build_ft_dataset(uo, tiles, thm, tvm, pals)
            g = ft.KeyframeTiler.__new__(ft.KeyframeTiler)
            g.kdt, g.use_wavelets, g.gamma = kt, True, -1
            got = g.do_frame_tiling(frames)
            kt.close()
            o = oracle.frame_tiling(frames, ods, ot, op, oa)
            assert np.array_equal(got[4].view(np.uint32), o[4].view(np.uint32)), q
            for a, b in zip(got[:4], o[:4]):
                assert np.array_equal(a, b), (q, int(np.count_nonzero(a != b)))
    finally:
        gds.kdt.close()

"""The benchmarked FrameTiling batch and the BASELINE C5 workload at full size, against the CPU restatement.

* C3 (the bench step): one 24-frame 1080p keyframe = 777,600 frame tiles through ONE
  tiler_frame_tiling call against a 64k tileset x 4 mirrors.  At this size the flat tiles are grouped last
  (nn_frame_tiling_dev): a stable permutation, shortlist workgroups made of flat tiles only (3 k-steps), the mixed
  workgroup at the boundary and the scatter back.  A sample that covers random tiles, flat tiles, the whole mixed
  workgroup and the last workgroup is checked against ANN 1.1.2's kd-tree search restated (oracle/ann_kdtree.c).
* C5: a 4K frame (129,600 tiles, grouped the same way) against 256k tiles x 4 mirrors = 1,048,576 candidates.
* Tier 2 at scale: a C3-size tileset in which every tile has 15 identical copies and frame tiles that are
  near-copies of tileset tiles, so nearly every query's lane lists fill with equal keys and the query goes to tier
  2 (main.pas:4027 must return for any input): bit-exact, no exhaustive scan, and at most 10x the time of a regular
  C3 keyframe measured in the same test.
References: DoFrameTiling main.pas:3992-4047, PrepareFrameTiling.DoPsyV 3883-3919, ANN call main.pas:4027.
"""
import time

import numpy as np
import pytest

from tiler_amd import synth

pytestmark = pytest.mark.gpu

WG_QUERIES = 512  # orbit shortlist workgroup: 8 waves x 2 query blocks x 32 (orbit.hip ORB_NW, QB)


def _flat_layout(rgb):
    """The grouping nn_frame_tiling_dev builds on the device: non-flat tiles first, flat ones after, each in tile
    order; returns (flat mask, permuted order, first all-flat workgroup)."""
    flat = np.all(rgb == rgb[:, :1], axis=1)
    order = np.concatenate([np.nonzero(~flat)[0], np.nonzero(flat)[0]])
    others = int((~flat).sum())
    return flat, order, -(-others // WG_QUERIES)


def _sample(rng, rgb, n_rand, n_flat, tail):
    flat, order, wf0 = _flat_layout(rgb)
    Q = rgb.shape[0]
    fl = np.nonzero(flat)[0]
    parts = [rng.choice(Q, n_rand, replace=False), rng.choice(fl, min(n_flat, fl.size), replace=False),
             order[max(0, (wf0 - 1) * WG_QUERIES):wf0 * WG_QUERIES],  # the mixed workgroup (last others, first flats)
             order[-tail:]]                                           # the last workgroup
    return np.unique(np.concatenate(parts)), flat, wf0


def _check_items(g, o, pick):
    assert np.array_equal(np.asarray(g[4])[pick].view(np.uint32), o[4].view(np.uint32)), "distance mismatch"
    for name, a, b in zip(("tile", "pal", "hmirror", "vmirror"), g[:4], o[:4]):
        a = np.asarray(a)[pick]
        assert np.array_equal(a, b), f"{name}: {np.count_nonzero(a != b)} of {pick.size} sampled items differ"


def _frame_tiling(kt, frames):
    t0 = time.perf_counter()
    g = kt.do_frame_tiling(frames)
    return g, time.perf_counter() - t0, kt.kdt.stats()


@pytest.mark.timeout(900)
def test_c3_keyframe_batch_flat_grouped_vs_ann(gpu, oracle):
    """The bench's step: 24 x 32,400 tiles in one call; >= 3,000 sampled items (>= 500 flat, the mixed and the
    last shortlist workgroup) equal the restated ANN search's tile, palette, mirror flags and distance."""
    from tiler_amd.frame_tiling import KeyframeTiler
    wl = synth.make_workload(3, 1920, 1080, 24, 65536, n_palettes=128)
    rgb = wl.frame_rgb.reshape(-1, 64)
    assert rgb.shape[0] == 777600
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    g, _, st = _frame_tiling(kt, rgb)
    kt.finish_frame_tiling()
    pick, flat, wf0 = _sample(np.random.default_rng(7), rgb, 2000, 600, 512)
    assert pick.size >= 3000 and flat[pick].sum() >= 500
    assert st["orbit_search"] == 1 and st["tie_order"] == 0
    wgs = -(-rgb.shape[0] // WG_QUERIES)
    assert st["flat_queries"] == rgb.shape[0] - wf0 * WG_QUERIES > 0  # the flat-only workgroups ran
    assert st["exhaustive_queries"] == 0
    used = synth.used_one_palette(wl.tile_pal, 128)
    ods, ot, op, oa = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    o = oracle.frame_tiling(rgb[pick], ods, ot, op, oa)
    _check_items(g, o, pick)
    assert wf0 < wgs


@pytest.mark.timeout(900)
def test_c5_frame_batch_flat_grouped_vs_ann(gpu, oracle):
    """C5: a 4K frame (129,600 tiles, >= 8,192 so grouped) against 1,048,576 candidates; >= 1,200 sampled items
    incl. flat tiles, the mixed and the last workgroup, against the restated ANN search."""
    from tiler_amd.frame_tiling import KeyframeTiler
    rng = np.random.default_rng(57)
    P, T = 128, 262144
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    tile_pal = rng.integers(0, P, T).astype(np.int32)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
    rgb = synth.frame_tiles(rng, 480 * 270)
    kt = KeyframeTiler(tiles, thm, tvm, pals, ds)
    g, _, st = _frame_tiling(kt, rgb)
    rows = kt.rows
    kt.finish_frame_tiling()
    pick, flat, wf0 = _sample(np.random.default_rng(8), rgb, 500, 300, 256)
    assert pick.size >= 1200 and flat[pick].sum() >= 300
    assert st["orbit_groups"] == T and st["tie_order"] == 0
    assert st["flat_queries"] == rgb.shape[0] - wf0 * WG_QUERIES > 0
    assert st["exhaustive_queries"] == 0
    o = oracle.frame_tiling(rgb[pick], rows, ds.tile_of, ds.pal_of, ds.attrs)
    _check_items(g, o, pick)


def _near_copy_frames(rng, tiles, pals, tile_pal, n, noise=2):
    """Frame tiles that are near-copies of tileset tiles: a random tile in a random orientation rendered with its
    palette, every channel moved by at most `noise`."""
    t = rng.integers(0, tiles.shape[0], n)
    pt = tiles[t].reshape(n, 8, 8)
    h = rng.random(n) < 0.5
    v = rng.random(n) < 0.5
    pt[h] = pt[h][:, :, ::-1]
    pt[v] = pt[v][:, ::-1, :]
    col = pals[tile_pal[t]][np.arange(n)[:, None], pt.reshape(n, 64)]
    ch = np.stack([(col >> s) & 255 for s in (0, 8, 16)], -1) + rng.integers(-noise, noise + 1, (n, 64, 3))
    ch = np.clip(ch, 0, 255)
    return synth.rgb_pack(ch[..., 0], ch[..., 1], ch[..., 2]).astype(np.int32)


@pytest.mark.timeout(900)
def test_tier2_flood_c3_bounded_and_exact(gpu, oracle):
    """Adversarial C3-size input: 4,096 distinct tiles x 16 identical copies (65,536 tiles, 262,144 candidates) and a
    keyframe of 24 x 32,400 near-copy frame tiles.  Every copy ties, the shortlist's lane lists (4 sub-blocks) fill
    with equal keys and the query goes to tier 2; the orbit tier 2 scores any number of candidates per query, so no
    query reaches the exhaustive scan, the call stays within 10x a regular C3 keyframe's, and a sample of 2,000
    queries equals the restated ANN search (its first-found copy among the 16)."""
    from tiler_amd.frame_tiling import KeyframeTiler
    # the regular C3 keyframe's time in the same process (reference for the bound)
    wl = synth.make_workload(3, 1920, 1080, 24, 65536, n_palettes=128)
    kt = KeyframeTiler(wl.tiles, wl.thm, wl.tvm, wl.palettes, wl.ds)
    _frame_tiling(kt, wl.frame_rgb.reshape(-1, 64))
    _, t_reg, st_reg = _frame_tiling(kt, wl.frame_rgb.reshape(-1, 64))
    kt.finish_frame_tiling()

    rng = np.random.default_rng(61)
    P, U, R = 128, 4096, 16
    pals = synth.palettes(rng, P)
    base, bhm, bvm = synth.tileset(rng, U)
    bpal = rng.integers(0, P, U).astype(np.int32)
    tiles, thm, tvm, tile_pal = (np.tile(a, (R,) + (1,) * (a.ndim - 1)) for a in (base, bhm, bvm, bpal))
    ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
    rgb = _near_copy_frames(rng, base, pals, bpal, 24 * 32400)
    kt = KeyframeTiler(tiles, thm, tvm, pals, ds)
    _frame_tiling(kt, rgb)
    g, t_adv, st = _frame_tiling(kt, rgb)
    rows = kt.rows
    kt.finish_frame_tiling()
    print(f"regular C3 keyframe {t_reg * 1e3:.1f} ms (tier 2: {st_reg['fallback_queries']}), flood "
          f"{t_adv * 1e3:.1f} ms (tier 2: {st['fallback_queries']}, tier 3: {st['exhaustive_queries']})")
    assert st["fallback_queries"] > rgb.shape[0] // 2, st
    assert st["exhaustive_queries"] == 0, st
    assert t_adv <= 10 * t_reg, (t_adv, t_reg)
    pick = np.random.default_rng(9).choice(rgb.shape[0], 2000, replace=False)
    o = oracle.frame_tiling(rgb[pick], rows, ds.tile_of, ds.pal_of, ds.attrs)
    _check_items(g, o, pick)

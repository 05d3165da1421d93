"""GPU parity of palette generation: tiler_quantize_palettes (QuantizePalette with DLv3 for
every (keyframe, palette) pair at once, CompareCMULHS order) bit-exact against the CPU restatement
(oracle/palette.c) -- palettes, use counts and DLv3 colour-table sizes -- on textured / gradient / flat tiles,
empty pairs, pairs with fewer colours than the palette, skipped (inactive / out-of-range) tiles and lookup bpc
4..8.  The oracle is unpinned against the reference DLL (quantizer.c is not buildable here)."""
import numpy as np
import pytest

from tiler_amd import synth
from tiler_amd.palette import quantize_palettes

pytestmark = pytest.mark.gpu


def _case(seed, kf_frames, q, P, flat_share=0.0):
    rng = np.random.default_rng(seed)
    tiles = [synth.keyframe_frames(rng, f, q).reshape(-1, 64) for f in kf_frames]
    pal_of = [rng.integers(0, P, t.shape[0]) + k * P for k, t in enumerate(tiles)]
    rgb = np.concatenate(tiles)
    if flat_share:
        flat = rng.random(rgb.shape[0]) < flat_share
        rgb[flat] = rgb[flat, :1]
    return rgb, np.concatenate(pal_of).astype(np.int32), len(kf_frames) * P


def _check(oracle, rgb, pal_of, pairs, bpc=7, active=None):
    g_pal, g_uc, g_h = quantize_palettes(rgb, pal_of, pairs, 16, bpc, active)
    o_pal, o_uc, o_h = oracle.quantize_palettes(rgb, pal_of, pairs, 16, bpc, active)
    assert np.array_equal(g_uc, o_uc)
    assert np.array_equal(g_h, o_h)
    bad = np.nonzero(np.any(g_pal != o_pal, 1))[0]
    assert bad.size == 0, (bad[:5], g_pal[bad[:2]], o_pal[bad[:2]])
    return g_h


def test_quantize_two_keyframes(gpu, oracle):
    rgb, pal_of, pairs = _case(1, (3, 2), 120, 6)
    h = _check(oracle, rgb, pal_of, pairs)
    assert h.max() > 1000  # textured tiles: the O(n^2) passes are exercised


def test_quantize_many_pairs(gpu, oracle):
    """1024 (keyframe, palette) pairs in one call, the clip-level form: the per-pair arrays of the workspace
    (use counts, segments, run count) are sized for every pair (an undersized carve once put the palette
    output past the end of the allocation at P >= 1024)."""
    rgb, pal_of, pairs = _case(11, (2, 2), 2048, 512)
    h = _check(oracle, rgb, pal_of, pairs)
    assert pairs == 1024 and (h > 0).sum() > 1000


@pytest.mark.parametrize("bpc", [4, 5, 6, 8])
def test_quantize_bpc(gpu, oracle, bpc):
    rgb, pal_of, pairs = _case(2 + bpc, (2,), 100, 4)
    _check(oracle, rgb, pal_of, pairs, bpc)


def test_quantize_edges(gpu, oracle):
    rgb, pal_of, pairs = _case(7, (2, 2), 60, 5, flat_share=0.6)
    pal_of[pal_of == 3] = 4       # pair 3 empty
    pal_of[::17] = 99             # out of range: skipped
    few = pal_of == 6             # pair 6: a handful of flat colours (fewer than 16)
    rgb[few] = np.int32(0x102030) + (np.arange(few.sum()) % 5)[:, None].astype(np.int32)
    active = (np.arange(rgb.shape[0]) % 11 != 0).astype(np.uint8)
    h = _check(oracle, rgb, pal_of, pairs, 7, active)
    assert h[3] == 0 and 0 < h[6] < 16


def test_quantize_clustered_long_recount_lists(gpu, oracle):
    """Few dominant colours with small noise: many entries share a nearest neighbour, so the merges' recount
    lists are long (the batched recount_next over many entries at once)."""
    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, (6, 3))
    n = 1500
    px = np.clip(base[rng.integers(0, 6, (n, 64))] + rng.integers(-10, 11, (n, 64, 3)), 0, 255).astype(np.int32)
    rgb = px[..., 0] | (px[..., 1] << 8) | (px[..., 2] << 16)
    pal_of = rng.integers(0, 3, n).astype(np.int32)
    _check(oracle, rgb, pal_of, 3)


@pytest.mark.parametrize("cap", [1, 3, 64])
def test_quantize_list_overflow(gpu, oracle, cap):
    """tiler_debug_dl3: with at most `cap` recount entries per LDS batch the merges' lists spill to the global
    overflow and run in several batches; palettes stay bit-exact."""
    from tiler_amd import load
    lib = load()
    rgb, pal_of, pairs = _case(5, (2,), 90, 3)
    assert lib.tiler_debug_dl3(cap) == 0
    try:
        _check(oracle, rgb, pal_of, pairs)
    finally:
        lib.tiler_debug_dl3(0)


@pytest.mark.parametrize("gamma", [-1, 0])
def test_lab_descriptor_bit_exact(gpu, oracle, gamma):
    """ComputeTilePsyVisFeatures(UseLAB) on the GPU (fdlibm exp / ln on device, detmath.hpp) equals the CPU
    restatement bit for bit, Haar and DCT."""
    from tiler_amd.psyv import psyv_batch
    rng = np.random.default_rng(20 + gamma)
    rgb = synth.frame_tiles(rng, 700)
    rgb[:5] = 0
    rgb[5:9] = 0xFFFFFF
    for wl in (True, False):
        g, _ = psyv_batch(rgb=rgb, flags=4 | (2 if wl else 0), gamma=gamma)
        o = oracle.psyv_lab_batch(rgb, gamma, wl)
        assert np.array_equal(g.view(np.uint64), o.view(np.uint64))


@pytest.mark.parametrize("n,k", [(3000, 8), (2500, 70), (200, 128), (50, 64)])
def test_kmeans_bit_exact(gpu, oracle, n, k):
    """Seeding, every Lloyd step, the final labels and centroids, and the iteration count equal the restatement's
    (k > 64 exercises the two-chunk assignment; n < k duplicates centres)."""
    from tiler_amd.palette import kmeans
    rng = np.random.default_rng(n + k)
    centers = rng.normal(0, 10, (max(2, k // 2), 192))
    X = centers[rng.integers(0, centers.shape[0], n)] + rng.normal(0, 3, (n, 192))
    gl, gc, gi = kmeans(X, k)
    ol, oc, oi = oracle.kmeans(X, k)
    assert gi == oi
    assert np.array_equal(gl, ol)
    assert np.array_equal(gc.view(np.uint64), oc.view(np.uint64))


def test_prepare_dither_tiles_bit_exact(gpu, oracle):
    from tiler_amd.palette import prepare_dither_tiles
    rgb = synth.keyframe_frames(np.random.default_rng(31), 3, 400).reshape(-1, 64)
    gl, gc, gi = prepare_dither_tiles(rgb, 16)
    ol, oc, oi = oracle.prepare_dither_tiles(rgb, 16)
    assert gi == oi and np.array_equal(gl, ol) and np.array_equal(gc, oc)
    zl, zc, _ = prepare_dither_tiles(rgb[:1], 16)  # fewer than two tiles: the reference's zero branch
    assert not zl.any() and not zc.any()


def test_generate_palettes_chain_bit_exact(gpu, oracle):
    """btnDitherClick's palette half over two keyframes on the GPU: DitheringPalIndex, palettes (DLv3 + CMULHS),
    centroids and the FinishQuantizePalette order equal the CPU chain's."""
    from tiler_amd.palette import generate_palettes
    rng = np.random.default_rng(41)
    frames = np.concatenate([synth.keyframe_frames(rng, 2, 300), synth.keyframe_frames(rng, 3, 300)])
    kf = np.array([0, 2, 5])
    g = generate_palettes(frames, kf, 8)
    o = oracle.generate_palettes(frames, kf, 8)
    for a, b, name in zip(g, o, ("palettes", "centroids", "dith", "use_count")):
        assert np.array_equal(a, b), name

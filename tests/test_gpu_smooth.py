"""GPU parity of Smooth (DoTemporalSmoothing main.pas:4071-4119) against the CPU restatement: items and
Smoothed flags bit-exact, including the 'PrevTMI^ := TMI^' branch that rewrites frame i-1."""
import numpy as np
import pytest

from tiler_amd import synth
from tiler_amd.smooth import smooth_keyframe

pytestmark = pytest.mark.gpu


def _tilemaps(rng, F, Q, T, P, repeat=0.6):
    """Tilemaps with temporal coherence: most positions keep (or nearly keep) the previous item."""
    tile = np.zeros((F, Q), np.int32)
    pal = np.zeros((F, Q), np.int32)
    hm = np.zeros((F, Q), np.uint8)
    vm = np.zeros((F, Q), np.uint8)
    tile[0] = rng.integers(0, T, Q)
    pal[0] = rng.integers(0, P, Q)
    hm[0] = rng.integers(0, 2, Q)
    vm[0] = rng.integers(0, 2, Q)
    for f in range(1, F):
        r = rng.random(Q)
        keep = r < repeat
        near = (r >= repeat) & (r < repeat + (1 - repeat) * 0.6)
        tile[f] = np.where(keep, tile[f - 1], rng.integers(0, T, Q))
        pal[f] = np.where(keep, pal[f - 1], rng.integers(0, P, Q))
        hm[f] = np.where(keep, hm[f - 1], rng.integers(0, 2, Q))
        vm[f] = np.where(keep, vm[f - 1], rng.integers(0, 2, Q))
        # near variants: the twin tile (T/2 apart, one pixel differs) or the twin palette (0 <-> 1)
        twin_t = (tile[f - 1] + T // 2) % T
        tile[f] = np.where(near & (r < repeat + 0.12), twin_t, tile[f])
        pal[f] = np.where(near & (r < repeat + 0.12), pal[f - 1], pal[f])
        other = near & (r >= repeat + 0.12)
        tile[f] = np.where(other, tile[f - 1], tile[f])
        pal[f] = np.where(other, np.where(pal[f - 1] == 0, 1, 0), pal[f])
        hm[f] = np.where(near, hm[f - 1], hm[f])
        vm[f] = np.where(near, vm[f - 1], vm[f])
    return tile, pal, hm, vm


@pytest.mark.parametrize("strength", [0.02, 0.08, 0.0])
def test_smooth_bit_exact(gpu, oracle, strength):
    rng = np.random.default_rng(31)
    F, Q, T, P = 12, 700, 120, 5
    palpix = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    # near-duplicate tiles (one pixel index apart) so |cmp| lands on both sides of Strength
    palpix[60:] = palpix[:60]
    palpix[60:, 5] = (palpix[60:, 5] + 1) % 16
    pals = synth.palettes(rng, P)
    pals[1] = pals[0] + 1
    tile, pal, hm, vm = _tilemaps(rng, F, Q, T, P)
    sm = np.zeros((F, Q), np.uint8)
    tmp = rng.integers(-1, 100, (F, Q)).astype(np.int32)
    g = smooth_keyframe(tile, pal, hm, vm, sm, palpix, pals, strength, tmpidx=tmp)
    o = oracle.smooth(tile, pal, hm, vm, sm, palpix, pals, strength, tmpidx=tmp)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)
    changed = int(np.count_nonzero(g[0] != tile))
    if strength > 0:
        assert g[4].sum() > 0 and changed > 0  # both branches exercised


def test_smooth_single_frame_is_identity(gpu):
    rng = np.random.default_rng(1)
    tile = rng.integers(0, 10, (1, 50)).astype(np.int32)
    z = np.zeros((1, 50), np.uint8)
    g = smooth_keyframe(tile, np.zeros_like(tile), z, z, z, rng.integers(0, 16, (10, 64)), synth.palettes(rng, 1))
    assert np.array_equal(g[0], tile)


@pytest.mark.timeout(600)
def test_smooth_c3_size(gpu, oracle):
    """Smooth at the C3 step's size: one keyframe of 24 frames x 32,400 positions (1080p), a 4,096-tile set with
    near-duplicate twins, 128 palettes, strength 0.04 (twice the default, so the one-pixel twins merge too): items
    and flags bit-exact against the restatement (which computes every compared descriptor; about a minute on the
    box's host).  The default 0.02 is checked at C5 size below."""
    rng = np.random.default_rng(2402)
    F, Q, T, P = 24, 32400, 4096, 128
    palpix = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    palpix[T // 2:] = palpix[:T // 2]
    palpix[T // 2:, 7] = (palpix[T // 2:, 7] + 1) % 16
    pals = synth.palettes(rng, P)
    pals[1] = pals[0] + 1
    tile, pal, hm, vm = _tilemaps(rng, F, Q, T, P)
    sm = np.zeros((F, Q), np.uint8)
    g = smooth_keyframe(tile, pal, hm, vm, sm, palpix, pals, 0.04)
    o = oracle.smooth(tile, pal, hm, vm, sm, palpix, pals, 0.04)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)
    assert g[4].sum() > 0


@pytest.mark.timeout(900)
def test_smooth_c5_size_default_strength(gpu, oracle):
    """BASELINE C5's Smooth: one 4K keyframe of 24 frames x 129,600 positions (DoTemporalSmoothing main.pas:4071-4119,
    positions independent, frames of one keyframe), 65,536 tiles with near-duplicate twins, 128 palettes whose first
    two differ by one RGB step, the DEFAULT strength 0.02.  The whole keyframe runs in one GPU call; 6,000 positions
    (columns of the [F][Q] maps: each column is its own chain) are checked bit for bit against the restatement."""
    rng = np.random.default_rng(2405)
    F, Q, T, P = 24, 480 * 270, 65536, 128
    palpix = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    palpix[T // 2:] = palpix[:T // 2]
    palpix[T // 2:, 7] = (palpix[T // 2:, 7] + 1) % 16
    pals = synth.palettes(rng, P)
    pals[1] = pals[0] + 1
    tile, pal, hm, vm = _tilemaps(rng, F, Q, T, P)
    sm = np.zeros((F, Q), np.uint8)
    g = smooth_keyframe(tile, pal, hm, vm, sm, palpix, pals, 0.02)
    cols = np.sort(rng.choice(Q, 6000, replace=False))
    sub = lambda a: np.ascontiguousarray(a[:, cols])  # noqa: E731
    o = oracle.smooth(sub(tile), sub(pal), sub(hm), sub(vm), sub(sm), palpix, pals, 0.02)
    for a, b in zip(g[:5], o[:5]):  # items and flags (tmpidx: None on both sides)
        assert np.array_equal(sub(a), b)
    assert g[4].sum() > 0 and sub(np.asarray(g[4])).sum() > 0  # the default strength does merge here

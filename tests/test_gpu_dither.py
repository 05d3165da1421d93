"""GPU parity of the Dither step per tile (DitherTile, Thomas Knoll mixing + PrepareTileMirrors) against the CPU
restatement: palette indices and mirror flags bit-exact, including palettes with duplicate colours and distinct
colours of equal luma (the reference QuickSort's tie order), palette sizes 4/8/16 and ragged tile counts."""
import numpy as np
import pytest

from tiler_amd import synth
from tiler_amd._lib import TilerError
from tiler_amd.dither import dither_tiles

pytestmark = pytest.mark.gpu


def _palettes(rng, P, size):
    pals = synth.rgb_pack(*rng.integers(0, 256, (3, P, size))).astype(np.int32)
    if size >= 16:
        for p in range(0, P, 2):  # every other palette with tie cases
            pals[p, 3] = pals[p, 1]
            pals[p, 5], pals[p, 6] = synth.rgb_pack(100, 100, 100), synth.rgb_pack(117, 90, 149)
            pals[p, 9], pals[p, 10] = synth.rgb_pack(200, 60, 30), synth.rgb_pack(135, 77, 53)
    return pals


@pytest.mark.parametrize("n,P,size", [(1, 1, 16), (5, 3, 16), (1000, 16, 16), (333, 8, 8), (130, 4, 4), (50, 3, 2), (10, 2, 1)])
def test_dither_bit_exact(gpu, oracle, n, P, size):
    rng = np.random.default_rng(n * 7 + size)
    rgb = synth.frame_tiles(rng, n)
    pal_of = rng.integers(0, P, n).astype(np.int32)
    pals = _palettes(rng, P, size)
    g = dither_tiles(rgb, pal_of, pals)
    o = oracle.dither_tiles_tk(rgb, pal_of, pals)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)


def test_dither_frame_sample(gpu, oracle):
    """A 720p frame's worth of tiles (14,400) on the GPU; a seeded sample of 1,500 re-checked on the CPU."""
    rng = np.random.default_rng(99)
    rgb = synth.frame_tiles(rng, 14400)
    pal_of = rng.integers(0, 32, 14400).astype(np.int32)
    pals = _palettes(rng, 32, 16)
    px, hm, vm = dither_tiles(rgb, pal_of, pals)
    idx = np.sort(rng.choice(14400, 1500, replace=False))
    opx, ohm, ovm = oracle.dither_tiles_tk(rgb[idx], pal_of[idx], pals)
    assert np.array_equal(px[idx], opx) and np.array_equal(hm[idx], ohm) and np.array_equal(vm[idx], ovm)
    assert int(px.max()) < 16


def test_dither_rejects_bad_input(gpu):
    rgb = np.zeros((2, 64), np.int32)
    with pytest.raises(TilerError):
        dither_tiles(rgb, np.array([0, 5], np.int32), np.zeros((2, 16), np.int32))   # palette index out of range
    with pytest.raises(TilerError):
        dither_tiles(rgb, np.array([0, 0], np.int32), np.zeros((2, 12), np.int32))   # palsize not a power of two


@pytest.mark.parametrize("mixed", [1, 2, 4, 8, 16])
def test_dither_yliluoma_bit_exact(gpu, oracle, mixed):
    """The Yliluoma branch (chkUseTK off; DeviseBestMixingPlanYliluoma's ASM_DBMP form, main.pas:1573-1826) at every
    cbxYilMix setting: palette indices and mirror flags equal to the restatement, tie palettes included."""
    rng = np.random.default_rng(500 + mixed)
    n, P = 400, 6
    rgb = synth.frame_tiles(rng, n)
    pal_of = rng.integers(0, P, n).astype(np.int32)
    pals = _palettes(rng, P, 16)
    g = dither_tiles(rgb, pal_of, pals, yliluoma_mix=mixed)
    o = oracle.dither_tiles_yl(rgb, pal_of, pals, mixed)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("size,mixed", [(5, 4), (8, 64), (1, 3), (16, 33)])
def test_dither_yliluoma_sizes(gpu, oracle, size, mixed):
    """Palette sizes that are not powers of two (the Yliluoma plan has no `c and (palsize - 1)` default), one entry,
    and mixed counts beyond the form's choices up to the 64 supported (lists of up to 126 entries)."""
    rng = np.random.default_rng(size * 100 + mixed)
    n, P = 64, 3
    rgb = synth.frame_tiles(rng, n)
    pal_of = rng.integers(0, P, n).astype(np.int32)
    pals = synth.rgb_pack(*rng.integers(0, 256, (3, P, size))).astype(np.int32)
    g = dither_tiles(rgb, pal_of, pals, yliluoma_mix=mixed)
    o = oracle.dither_tiles_yl(rgb, pal_of, pals, mixed)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)


def test_dither_yliluoma_rejects_bad_input(gpu):
    rgb = np.zeros((2, 64), np.int32)
    pal_of = np.array([0, 0], np.int32)
    for mixed in (-1, 65):
        with pytest.raises(TilerError):
            dither_tiles(rgb, pal_of, np.zeros((1, 16), np.int32), yliluoma_mix=mixed)
    with pytest.raises(TilerError):
        dither_tiles(rgb, pal_of, np.zeros((1, 17), np.int32), yliluoma_mix=4)   # more than 16 palette entries

"""GlobalTiling (DoGlobalTiling main.pas:4256-4370): host glue on CPU, the K-Modes merge pass on the GPU,
both against the CPU restatement."""
import numpy as np
import pytest

from tiler_amd import global_tiling as gt
from tiler_amd import synth


def _tiles(rng, T, P, dup=0.1):
    tiles, _, _ = synth.tileset(rng, T)
    base = tiles[: max(1, T // 20)]
    pick = rng.random(T) < dup
    tiles[pick] = base[rng.integers(0, base.shape[0], int(pick.sum()))]  # exact duplicates for MakeUnique
    # smooth-ish tiles so K-Modes has structure: blend toward a few prototypes
    protos = rng.integers(0, 16, (30, 64)).astype(np.uint8)
    near = rng.random(T) < 0.5
    src = protos[rng.integers(0, 30, int(near.sum()))]
    mask = rng.random(src.shape) < 0.8
    tiles[near] = np.where(mask, src, tiles[near])
    dith = rng.zipf(1.5, T) % P
    return tiles, dith.astype(np.int32)


def test_dataset_line_and_eqtc(oracle):
    rng = np.random.default_rng(1)
    tiles, _ = _tiles(rng, 200, 4)
    lines = gt.write_tile_dataset_line(tiles)
    for i in range(0, 200, 13):
        ref = np.zeros(80, np.uint8)
        oracle.lib().or_tile_dataset_line(tiles[i].ctypes.data_as(__import__("ctypes").c_void_p), 16,
                                          ref.ctypes.data_as(__import__("ctypes").c_void_p))
        assert np.array_equal(lines[i], ref)
    for n in (0, 1, 5, 100, 12345, 999999):
        assert gt.equal_quality_tile_count(n) == oracle.lib().or_eqtc(float(n))


def test_make_unique_and_reindex_match_oracle(oracle):
    import ctypes
    rng = np.random.default_rng(2)
    tiles, _ = _tiles(rng, 500, 4, dup=0.3)
    uc = rng.integers(1, 50, 500).astype(np.int32)
    pp, act, ucn, mi = gt.make_tiles_unique(tiles, np.ones(500, np.uint8), uc)
    opp = tiles.copy()
    oact = np.ones(500, np.uint8)
    ouc = uc.copy()
    omi = np.zeros(500, np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    oracle.lib().or_make_tiles_unique(500, p(opp), p(oact), p(ouc), p(omi))
    assert np.array_equal(pp, opp) and np.array_equal(act, oact) and np.array_equal(ucn, ouc)
    assert np.array_equal(mi, omi)
    idx = gt.reindex_tiles(act, ucn)
    oidx = np.zeros(500, np.int32)
    oracle.lib().or_reindex(500, p(oact), p(ouc), p(oidx))
    assert np.array_equal(idx, oidx)


@pytest.mark.gpu
def test_global_tiling_kmodes_pass_bit_exact(gpu, oracle):
    rng = np.random.default_rng(3)
    T, P = 3000, 6
    tiles, dith = _tiles(rng, T, P)
    g = gt.do_global_tiling(tiles, dith, P, desired=400)
    o = oracle.global_tiling(tiles, dith, P, desired=400)
    assert np.array_equal(g[4], o[4])          # cluster budget per bin
    assert np.array_equal(g[0], o[0])          # tiles (merged ones zeroed)
    assert np.array_equal(g[1], o[1])          # Active
    assert np.array_equal(g[2], o[2])          # UseCount
    assert np.array_equal(g[3], o[3])          # MergeIndex
    assert g[1].sum() < T                      # something merged

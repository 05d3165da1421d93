"""GPU parity of the mirror-orbit search path (tiler_amd/csrc/orbit.hip) against the CPU restatement.

The orbit path scores the 4 H/V mirrors of a tile (PrepareFrameTiling.DoPsyV emission order,
main.pas:3883-3919) with one MFMA pass; results must stay bit-identical to the exhaustive reference-order
scan: index, fp32 distance, lowest index on exact ties.
"""
import numpy as np
import pytest

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
    with gpu.KDTree(data) as kdt:
        gi, ge = kdt.search_batch(qs)
        st = kdt.stats()
    oi, oe = oracle.nn_batch(data, qs)
    assert np.array_equal(gi, oi), f"{np.count_nonzero(gi != oi)} index mismatches of {len(qs)}"
    assert np.array_equal(ge.view(np.uint32), oe.view(np.uint32))
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
    """Queries that ARE candidates (distance 0): symmetric tiles tie across mirrors -> lowest index."""
    rng, ods, *_ = _ft_rows(oracle, 33, 1200, 8)
    pick = rng.integers(0, ods.shape[0], 700)
    q = ods[pick].copy()
    st = _check(gpu, oracle, ods, q)
    assert st["exhaustive_queries"] == 0


def test_orbit_duplicate_tiles_force_overflow(gpu, oracle):
    """Many identical tiles (same palette) make equal-distance groups larger than the shortlists: the
    overflow tiers must still return the lowest-index winner."""
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

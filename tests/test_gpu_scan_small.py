"""The small-batch exact scan (the reference's per-tile ann_kdtree_search calls, coalesced by the library;
SURVEY.md 8(b); nn_scan_small_kernel + nn_scan_merge_kernel), bit-exact against the restated ANN search and the
lowest-index scan (nncheck, which also runs each batch through the MFMA tiers): batches of 1..64 queries, a prefix of
equal dimensions with coarse-grid values and duplicated rows (ties in ANN's order), rows at +inf distance, rows of
4..36 dimensions, and more than 256 candidates per workgroup at the 1,024-split cap.  (Round 5 also measured a
partial-distance pruning of this scan against these tests: exact, but no faster on PsyV rows -- DESIGN.md section 4.)"""
import numpy as np
import pytest

from nncheck import check_nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nq", [1, 3, 16, 64])
def test_scan_small_random(gpu, oracle, nq):
    rng = np.random.default_rng(100 + nq)
    data = rng.standard_normal((5000, 192)).astype(np.float32)
    q = data[rng.choice(5000, nq, replace=False)] + rng.standard_normal((nq, 192)).astype(np.float32) * 0.3
    check_nn(gpu, oracle, data, q)


def test_scan_small_flat_prefix_and_ties(gpu, oracle):
    """The first 32 dimensions equal in every row (the prefix bounds nothing), values on a coarse grid (many equal
    distances), duplicated rows (ties resolved by the tie order)."""
    rng = np.random.default_rng(7)
    base = (rng.integers(0, 3, (3000, 128)) * 0.5).astype(np.float32)
    data = np.concatenate([np.full((3000, 32), 0.25, np.float32), base], axis=1)
    data = np.concatenate([data, data[:1500]])
    q = data[rng.choice(data.shape[0], 40, replace=False)]
    check_nn(gpu, oracle, data, q)


def test_scan_small_infinite_distances(gpu, oracle):
    """Rows whose squares overflow to +inf inside the prefix or after it (NaN rows are out: what ANN returns around a
    NaN distance depends on its visit order, test_gpu_edges::test_nonfinite_dataset_builds_and_searches)."""
    rng = np.random.default_rng(8)
    data = rng.standard_normal((4000, 64)).astype(np.float32)
    data[::97, 5] = 3e19            # +inf inside the prefix
    data[3::101, 50] = -3e19        # +inf after it
    data[7::89, :] = 3e19           # every term +inf
    q = rng.standard_normal((20, 64)).astype(np.float32)
    check_nn(gpu, oracle, data, q)


@pytest.mark.parametrize("d", [4, 32, 36])
def test_scan_small_short_rows(gpu, oracle, d):
    rng = np.random.default_rng(9 + d)
    data = rng.standard_normal((6000, d)).astype(np.float32)
    check_nn(gpu, oracle, data, rng.standard_normal((17, d)).astype(np.float32))


def test_scan_small_several_rounds_per_thread(gpu, oracle):
    """300,000 candidates: more than 256 per workgroup at the 1,024-split cap, so the bound carries over rounds."""
    rng = np.random.default_rng(10)
    data = rng.standard_normal((300000, 48)).astype(np.float32)
    q = data[rng.choice(300000, 9, replace=False)] + 0.05
    check_nn(gpu, oracle, data, q)


@pytest.mark.parametrize("k", [1, 8])
def test_scan_small_orbit_index(gpu, oracle, k):
    """A mirror-orbit dataset (a tileset in its 4 orientations: PsyV rows that are exact signed permutations of their
    group's base row, 20 % symmetric tiles with identical mirrors): batches of up to 4 queries take nn_scan_orbit_kernel,
    which reads only the base rows and forms every member's values from them (larger ones the generic scan).  Batches of 1, 3, 16 and 64 queries (16 for k = 8),
    frame tiles and perturbed candidate rows (exact ties among a tile's mirrors), both tie orders."""
    from tiler_amd import synth
    rng = np.random.default_rng(31 + k)
    P, T = 16, 3000
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = gpu.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                          flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    with gpu.KDTree(rows) as kdt:
        assert kdt.stats()["orbit_groups"] > 0
    picks = rows[rng.choice(rows.shape[0], 64, replace=False)]
    qs = np.concatenate([picks[:32], picks[32:] + rng.standard_normal((32, 192)).astype(np.float32) * 0.01])
    for nq in ((1, 3, 16) if k == 8 else (1, 3, 16, 64)):
        check_nn(gpu, oracle, rows, qs[:nq], k=k)


def test_scan_small_k8_ties(gpu, oracle):
    """k = 8 small batches on a plain index whose rows come in groups of 4 identical copies at scattered positions
    (a flat tile's 4 orientations in a shuffled PrepareFrameTiling set): every copy must survive the per-thread,
    per-workgroup and merge lists in ANN's tie order.  The round-4 merge lost a copy (tools/k8_plain_check.py: 28 of
    256 frame tiles on the shuffled C3 rows): its per-lane K-lists over up to 16 splits were miscompiled on exact ties.
    The merge is now the wide cross-lane one (nn_scan_merge_kernel: one split per thread, k rounds of argmin over the
    split heads, no per-lane list), and the per-thread lists of the scan insert through kd_list_insert
    (test_gpu_list_ties.py places the copies in one old merge lane and in one scan thread on purpose)."""
    rng = np.random.default_rng(77)
    base = rng.standard_normal((6000, 192)).astype(np.float32)
    rows = np.concatenate([base, np.repeat(base[:1500], 3, axis=0)])[rng.permutation(6000 + 4500)]
    picks = base[rng.choice(1500, 16, replace=False)]
    qs = np.concatenate([picks[:8], picks[8:] + rng.standard_normal((8, 192)).astype(np.float32) * 0.05])
    for nq in (1, 3, 16):
        check_nn(gpu, oracle, rows, qs[:nq], k=8)

"""CPU tests of the oracle (the checker) against known answers and the reference's own asm.

Pins:
  - K-Modes dissimilarity / argmin / min-distance update: the reference's x86-64 asm (kmodes.pas:316-596)
    assembled here (oracle/_ref, when /root/reference is mounted) and its committed vectors
    (tests/golden/kmodes_asm_kat.npz) everywhere else;
  - descriptor: analytic known answers (orthonormal Haar, mirror identities, DCT structure);
  - ANN distance / selection: independent numpy fp32 restatement.
"""
import ctypes
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_kmodes_dissim_matches_reference_asm_fixture(oracle):
    kat = np.load(os.path.join(GOLD, "kmodes_asm_kat.npz"))
    for t in range(kat["counts"].size):
        n = int(kat["counts"][t])
        rows = kat["rows"][t, :n]
        item = kat["items"][t]
        bi, bd = oracle.km_get_min(rows, item)
        assert bi == kat["best_idx"][t] and bd == kat["best_dis"][t], t
        md = kat["md_in"][t, :n].copy()
        oracle.lib().or_km_update_min_distance(item.ctypes.data_as(ctypes.c_void_p), rows.ctypes.data_as(ctypes.c_void_p),
                                               n, md.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(md, kat["md_out"][t, :n]), t


def test_kmodes_dissim_matches_live_reference_asm(oracle):
    ref = oracle.ref_kmodes_lib()
    if ref is None:
        pytest.skip("reference asm not built here (no /root/reference): the committed fixture pins it")
    rng = np.random.default_rng(9)
    for _ in range(300):
        n = int(rng.integers(1, 30))
        rows = rng.integers(0, 256, (n, 80), dtype=np.uint8)
        item = rng.integers(0, 256, 80, dtype=np.uint8)
        ptrs = (ctypes.c_void_p * n)(*[rows[i].ctypes.data for i in range(n)])
        best = ctypes.c_uint64()
        bi = ref.ref_get_min(item.ctypes.data_as(ctypes.c_void_p), ptrs, ctypes.c_uint64(n), ctypes.byref(best))
        assert (bi, best.value) == oracle.km_get_min(rows, item)


def test_kmodes_dissim_sse_form_equals_restatement(oracle):
    """The oracle's SSE2 dissimilarity (argmin / min-distance loops) equals its scalar restatement of the asm."""
    rng = np.random.default_rng(19)
    f = oracle.lib().or_km_dissim_fast
    f.restype = ctypes.c_uint64
    for t in range(3000):
        hi = [2, 16, 256][t % 3]
        a = rng.integers(0, hi, 80, dtype=np.int64).astype(np.uint8)
        b = rng.integers(0, hi, 80, dtype=np.int64).astype(np.uint8)
        if t % 7 == 0:
            b = a.copy()
        assert f(a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p)) == oracle.km_dissim(a, b)


def test_kmodes_asm_quirk_differs_from_generic(oracle):
    """The executed asm covers only bytes {0,1*256,8,9*256,16..79} in its L1 term."""
    a = np.zeros(80, np.uint8)
    b = np.zeros(80, np.uint8)
    b[2] = 5  # byte 2: counted as a mismatch only
    assert oracle.km_dissim(a, b) == 2048
    b[2] = 0
    b[1] = 3  # byte 1: weight 256
    assert oracle.km_dissim(a, b) == 2048 + 768
    b[1] = 0
    b[20] = 7
    assert oracle.km_dissim(a, b) == 2048 + 7
    b[20] = 0
    b[0] = 200  # pabsb of int8(-200)= |56|
    assert oracle.km_dissim(a, b) == 2048 + 56


def test_randint_delphi_lcg(oracle):
    seed = 0x42381337
    exp_seed = (seed * 0x08088405 + 1) & 0xFFFFFFFF
    r, s = oracle.randint(1000, seed)
    assert s == exp_seed and r == (exp_seed * 1000) >> 32


def test_eqtc_rounding(oracle):
    import math
    for n in (0, 1, 2, 3, 10, 100, 960, 12345, 1 << 20):
        v = math.sqrt(n) * (math.log(1 + n) / math.log(2))
        assert oracle.lib().or_eqtc(float(n)) == round(v)  # Python round = half-even like FPC Round


def _haar_np(x):
    """independent numpy WaveletGS (main.pas:2805-2840)"""
    f = 1.0 / np.sqrt(2.0)
    o = x.reshape(8, 8).copy()
    n = 8
    while n >= 2:
        blk = o[:n, :n]
        h = n // 2
        tx = np.empty_like(blk)
        tx[:, :h] = (blk[:, 0::2] + blk[:, 1::2]) * f
        tx[:, h:] = (blk[:, 0::2] - blk[:, 1::2]) * f
        ty = np.empty_like(blk)
        ty[:h, :] = (tx[0::2, :] + tx[1::2, :]) * f
        ty[h:, :] = (tx[0::2, :] - tx[1::2, :]) * f
        o[:n, :n] = ty
        n //= 2
    return o.reshape(64)


def _yuv_np(rgb):
    r = (rgb & 255) / 255.0
    g = ((rgb >> 8) & 255) / 255.0
    b = ((rgb >> 16) & 255) / 255.0
    y = (2126.0 * r + 7152.0 * g + 722.0 * b) / 10000.0
    return y, (b - y) * (0.5 / (1.0 - 722.0 / 10000.0)), (r - y) * (0.5 / (1.0 - 2126.0 / 10000.0))


def test_psyv_haar_matches_independent_numpy(oracle):
    rng = np.random.default_rng(3)
    from tiler_amd import synth
    for t in synth.frame_tiles(rng, 50):
        d = oracle.psyv(rgb=t, flags=2)
        exp = np.concatenate([_haar_np(c) for c in _yuv_np(t)])
        assert np.array_equal(d, exp)


def test_psyv_flat_tile_is_dc_only(oracle):
    t = np.full(64, 0x336699, np.int32)
    d = oracle.psyv(rgb=t, flags=2)
    y, u, v = _yuv_np(t[:1])
    for c, val in enumerate((y[0], u[0], v[0])):
        assert d[c * 64] == pytest.approx(8 * val, rel=1e-14)
        assert np.all(d[c * 64 + 1:(c + 1) * 64] == 0.0)


def test_psyv_haar_parseval_and_mirrors(oracle):
    rng = np.random.default_rng(4)
    from tiler_amd import synth
    for t in synth.frame_tiles(rng, 20):
        d = oracle.psyv(rgb=t, flags=2)
        ys = np.concatenate(_yuv_np(t))
        assert np.sum(d * d) == pytest.approx(np.sum(ys * ys), rel=1e-12)
        hm = synth.hflip(t[None])[0]
        vm = synth.vflip(t[None])[0]
        assert np.array_equal(oracle.psyv(rgb=t, flags=2 | 16), oracle.psyv(rgb=hm, flags=2))
        assert np.array_equal(oracle.psyv(rgb=t, flags=2 | 32), oracle.psyv(rgb=vm, flags=2))


def test_psyv_dct_structure(oracle):
    """DCT branch: sequential sums against gDCTLut, Q-weighting 4/sqrt(q), cUVRatio (main.pas:3075-3175)."""
    rng = np.random.default_rng(5)
    from tiler_amd import synth
    lut = np.ctypeslib.as_array(ctypes.cast(oracle.lib().or_dct_lut(), ctypes.POINTER(ctypes.c_double)), (4096,))
    t = synth.frame_tiles(rng, 1)[0]
    d = oracle.psyv(rgb=t, flags=0)
    dq = oracle.psyv(rgb=t, flags=8)
    ys = _yuv_np(t)
    ratio = np.ones(64)
    ratio[:8] = np.sqrt(0.5)
    ratio[::8] = np.sqrt(0.5)
    ratio[0] = 0.5
    for c in range(3):
        for o in range(64):
            z = 0.0
            for k in range(64):
                z += ys[c][k] * lut[o * 64 + k]
            assert d[c * 64 + o] == z * ratio[o]
    assert dq[0] == pytest.approx(d[0] * 4.0 / 4.0)  # luma (0,0): q = 16 -> 4/sqrt(16) = 1
    assert dq[1] == pytest.approx(d[1] * 4.0 / np.sqrt(11.0))


def test_psyv_golden_fixture(oracle):
    g = np.load(os.path.join(GOLD, "psyv_kat.npz"))
    for i, f in enumerate(g["flags_rgb"]):
        for j, t in enumerate(g["rgb"]):
            assert np.array_equal(oracle.psyv(rgb=t, flags=int(f)), g["out_rgb"][i, j])
    for i, f in enumerate(g["flags_pal"]):
        for j, t in enumerate(g["palpix"]):
            assert np.array_equal(oracle.psyv(palpix=t, pal=g["pal"], flags=int(f)), g["out_pal"][i, j])


def _np_dist(q, data):
    """independent fp32 sequential restatement of ANN's leaf distance"""
    acc = np.zeros(data.shape[0], np.float32)
    for k in range(data.shape[1]):
        t = (q[k] - data[:, k]).astype(np.float32)
        acc = (acc + (t * t).astype(np.float32)).astype(np.float32)
    return acc


def test_nn_and_knn_semantics(oracle):
    rng = np.random.default_rng(6)
    data = rng.normal(0, 1, (700, 24)).astype(np.float32)
    data[350:400] = data[0:50]  # exact ties
    for i in range(60):
        q = data[i] + (0 if i % 2 else rng.normal(0, 0.1, 24).astype(np.float32))
        d = _np_dist(q.astype(np.float32), data)
        idx, err = oracle.nn(data, q)
        assert idx == int(np.argmin(d)) and np.float32(err) == d.min()  # argmin = lowest index among ties
        ki, ke = oracle.knn(data, q, 8)
        order = np.lexsort((np.arange(d.size), d))[:8]
        assert np.array_equal(ki, order) and np.array_equal(ke, d[order])


def test_knn_more_than_n(oracle):
    data = np.arange(12, dtype=np.float32).reshape(3, 4)
    ki, ke = oracle.knn(data, data[1], 5)
    assert list(ki[:3]) == [1, 0, 2] and list(ki[3:]) == [-1, -1]


def test_ft_dataset_emission_order(oracle):
    """DoPsyV order: palette asc, tile asc, vmir, hmir; attrs H=1 V=2; mirror xor canonical flags."""
    from tiler_amd import synth
    rng = np.random.default_rng(7)
    tiles, thm, tvm = synth.tileset(rng, 40)
    used = (rng.random((3, 40, 4)) < 0.3).astype(np.uint8)
    ds = synth.ft_dataset_from_used(used, thm, tvm)
    pals = synth.palettes(rng, 3)
    od, ot, op, oa = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    assert np.array_equal(ot, ds.tile_of) and np.array_equal(op, ds.pal_of) and np.array_equal(oa, ds.attrs)
    for r in range(0, ot.size, 7):
        fl = 1 | 2 | int(ds.psyv_flags[r])
        exp = oracle.psyv(palpix=tiles[ot[r]], pal=pals[op[r]], flags=fl).astype(np.float32)
        assert np.array_equal(exp, od[r])


def test_prepare_tile_mirrors_canonical():
    from tiler_amd import synth
    t = np.zeros((1, 64), np.uint8)
    t[0, 7 * 8 + 7] = 15  # bottom-right quadrant heaviest -> H and V flips
    out, hm, vm = synth.prepare_tile_mirrors(t)
    assert hm[0] == 1 and vm[0] == 1 and out[0, 0] == 15
    t = np.zeros((1, 64), np.uint8)
    _, hm, vm = synth.prepare_tile_mirrors(t)  # all equal -> first (no mirror)
    assert hm[0] == 0 and vm[0] == 0


def test_ann_kdtree_baseline_exact_distances(oracle):
    """The CPU baseline's ANN-style kd-tree (oracle/ann_kdtree.c) returns the exhaustive scan's distance
    bit for bit (eps = 0), including duplicate rows, flat queries and an empty tree; among equal distances
    it may pick another index (ANN's visit order)."""
    from tiler_amd import synth
    rng = np.random.default_rng(12)
    tiles, thm, tvm = synth.tileset(rng, 600)
    pals = synth.palettes(rng, 4)
    used = synth.used_one_palette(rng.integers(0, 4, 600).astype(np.int32), 4)
    rows, *_ = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    q = np.concatenate([oracle.psyv_batch(400, rgb=synth.frame_tiles(rng, 400), flags=2).astype(np.float32),
                        rows[::37]])
    kd = oracle.KDTree(rows)
    ki, ke = kd.search_batch(q, threads=4)
    si, se = oracle.nn_batch(rows, q, threads=4)
    assert np.array_equal(ke.view(np.uint32), se.view(np.uint32))
    d = ((rows[ki].astype(np.float64) - q) ** 2).sum(1)
    assert np.allclose(d, se, rtol=1e-5)
    assert 0 < kd.visited < len(q) * rows.shape[0]
    kd.close()
    e = oracle.KDTree(np.zeros((0, 192), np.float32))
    i, _ = e.search_batch(q[:3], threads=1)
    assert (i == -1).all()


def test_fast_colour_division_is_exact(tmp_path):
    """psyv.hip's gamma = -1 query path replaces x / 10000.0 by a reciprocal multiply + one fma correction;
    it must equal the IEEE division for every colour sum of the domain (2^24 cases, oracle/check_fastdiv.c)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    exe = tmp_path / "check_fastdiv"
    src = os.path.join(os.path.dirname(__file__), "..", "oracle", "check_fastdiv.c")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), src, "-lm"], check=True)
    tot, bad = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert tot == 1 << 24 and bad == 0


def test_div255_identity():
    """psyv_dev.hpp div255: fma(fma(-q0, 255, r), RN(1/255), q0) with q0 = RN(r * RN(1/255)) equals the IEEE
    division r / 255.0 for every byte (the gamma = -1 LUT row), emulated exactly with rationals."""
    from fractions import Fraction as F
    inv = 1.0 / 255.0
    for r in range(256):
        q0 = float(F(r) * F(inv))
        res = float(F(r) - F(q0) * 255)
        assert float(F(res) * F(inv) + F(q0)) == r / 255.0, r


def test_orbit_pack_table_matches_orbit_map():
    """orbit_map_gen.hpp's PACK words (the fused query kernel's transform table) decode to the orbit map the
    generator derives from the Haar mirror permutations, for all three components (component independence)."""
    import os
    import re
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import gen_orbit_map
    src, wts, cnt = gen_orbit_map.build_map()
    txt = open(os.path.join(root, "tiler_amd", "csrc", "orbit_map_gen.hpp")).read()
    pack = [int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", txt.split("PACK[64]")[1])]
    assert len(pack) == 64
    for x in range(4):
        for j in range(16):
            w = pack[x * 16 + j]
            n = w >> 28
            for c in range(3):
                k = x * 48 + c * 16 + j
                assert n == cnt[k]
                for t in range(n):
                    assert ((w >> (6 * t)) & 63) + 64 * c == src[k][t]
                    assert (-1 if (w >> (24 + t)) & 1 else 1) == wts[k][t]

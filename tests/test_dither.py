"""Dither step per tile (DitherTile, Thomas Knoll mixing main.pas:1828-1875 / 1998-2055, PrepareTileMirrors
main.pas:4049-4069): the CPU restatement (oracle/dither_tk.c) against known answers and an independent Python
evaluation.  No reference fixture exists for this step (no FPC; yakmo / palettes are not in the reference):
parity against the reference binary is unpinned; the order of operations is restated from the source."""
import numpy as np
import pytest

from tiler_amd import synth

MAP = [0, 48, 12, 60, 3, 51, 15, 63, 32, 16, 44, 28, 35, 19, 47, 31, 8, 56, 4, 52, 11, 59, 7, 55, 40, 24, 36, 20,
       43, 27, 39, 23, 2, 50, 14, 62, 1, 49, 13, 61, 34, 18, 46, 30, 33, 17, 45, 29, 10, 58, 6, 54, 9, 57, 5, 53,
       42, 26, 38, 22, 41, 25, 37, 21]


def _tdiv(a, b):  # Pascal div (truncation toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _py_plan(pal, col):
    """DeviseBestMixingPlanThomasKnoll in Python ints, then the reference QuickSort (kmodes.pas:89-136)."""
    rgb = [(c & 255, (c >> 8) & 255, (c >> 16) & 255) for c in pal]
    luma = [r * 2126 + g * 7152 + b * 722 for r, g, b in rgb]
    s = (col & 255, (col >> 8) & 255, (col >> 16) & 255)
    e = [0, 0, 0]
    lst = []
    for c in range(64):
        t = [s[k] + _tdiv(e[k] * 9, 100) for k in range(3)]
        l1 = t[0] * 2126 + t[1] * 7152 + t[2] * 722
        best, chosen = None, c & (len(pal) - 1)
        for i, (r, g, b) in enumerate(rgb):
            ld = _tdiv(l1 - luma[i], 10000)
            pen = ((t[0] - r) ** 2) * 13 + ((t[1] - g) ** 2) * 13 + ((t[2] - b) ** 2) * 13 + (ld * ld << 5)
            if best is None or pen < best:
                best, chosen = pen, i
        lst.append(chosen)
        for k in range(3):
            e[k] += s[k] - rgb[chosen][k]

    def qs(a, first, last):
        if last <= first:
            return
        while True:
            i, j, p = first, last, (first + last) >> 1
            while True:
                while luma[a[i]] < luma[a[p]]:
                    i += 1
                while luma[a[j]] > luma[a[p]]:
                    j -= 1
                if i <= j:
                    a[i], a[j] = a[j], a[i]
                    if p == i:
                        p = j
                    elif p == j:
                        p = i
                    i += 1
                    j -= 1
                if i > j:
                    break
            if first < j:
                qs(a, first, j)
            first = i
            if i >= last:
                break
    qs(lst, 0, 63)
    return np.asarray(lst, np.uint8), luma


def _palette(rng, size=16, ties=False):
    pal = synth.rgb_pack(*rng.integers(0, 256, (3, size)))
    if ties:  # duplicate colours and distinct colours of equal luma -> the sort's tie order matters
        pal[3] = pal[1]                                            # duplicate colour
        pal[5] = synth.rgb_pack(100, 100, 100)                     # equal luma, distinct colours:
        pal[6] = synth.rgb_pack(117, 90, 149)                      # 17*2126 - 10*7152 + 49*722 = 0
        pal[9] = synth.rgb_pack(200, 60, 30)
        pal[10] = synth.rgb_pack(135, 77, 53)                      # -65*2126 + 17*7152 + 23*722 = 0
    return pal.astype(np.int32)


@pytest.mark.parametrize("ties", [False, True])
def test_tk_plan_matches_python(oracle, ties):
    rng = np.random.default_rng(21 + ties)
    for _ in range(6):
        pal = _palette(rng, ties=ties)
        for col in synth.rgb_pack(*rng.integers(0, 256, (3, 20))):
            o = oracle.tk_plan(pal, int(col))
            p, luma = _py_plan([int(c) for c in pal], int(col))
            assert np.array_equal(o, p)
            if ties:
                assert luma[5] == luma[6] and luma[9] == luma[10]
            assert all(luma[a] <= luma[b] for a, b in zip(o[:-1], o[1:]))   # sorted by luma


def test_tk_plan_known_answers(oracle):
    pal = _palette(np.random.default_rng(4))
    for i in (0, 7, 15):
        assert np.all(oracle.tk_plan(pal, int(pal[i])) == i)   # an exact palette colour: never any error
    gray = synth.rgb_pack(*([np.arange(16) * 17] * 3)).astype(np.int32)
    lst = oracle.tk_plan(gray, int(synth.rgb_pack(25, 25, 25)))  # between entries 1 (17) and 2 (34)
    assert set(lst.tolist()) <= {1, 2} and 0 < int((lst == 2).sum()) < 64


def test_dither_tiles_composition(oracle):
    """or_dither_tiles_tk = per-pixel plan -> cDitheringMap pick -> PrepareTileMirrors."""
    rng = np.random.default_rng(8)
    pals = np.stack([_palette(rng, ties=k % 2 == 1) for k in range(4)])
    rgb = synth.frame_tiles(rng, 12)
    pal_of = rng.integers(0, 4, 12).astype(np.int32)
    px, hm, vm = oracle.dither_tiles_tk(rgb, pal_of, pals)
    raw = np.array([[oracle.tk_plan(pals[pal_of[t]], int(rgb[t, k]))[MAP[k]] for k in range(64)] for t in range(12)],
                   np.uint8)
    cpx, chm, cvm = synth.prepare_tile_mirrors(raw)
    assert np.array_equal(px, cpx.reshape(12, 64)) and np.array_equal(hm, chm) and np.array_equal(vm, cvm)


def test_video_from_frames_host_logic(oracle):
    """synth.video_from_frames (the Load -> Dither hand-over of encoder.load_and_dither) with the restatements:
    keyframe starts from the split, palettes stacked per keyframe, tiles in canonical orientation."""
    rng = np.random.default_rng(12)
    tm_w, tm_h = 6, 4
    frames, starts = synth.shot_frames(rng, 10, tm_w, tm_h, shot_len=(3, 4))
    kf, nkf = oracle.find_keyframes(oracle.interframe_corr_batch(frames, tm_w, tm_h), 10, tm_w * tm_h)
    pals = np.stack([synth.palettes(np.random.default_rng(k), 4) for k in range(nkf)])
    v = synth.video_from_frames(frames, kf, pals, oracle.dither_tiles_tk)
    assert v.kf_start[0] == 0 and v.kf_start[-1] == 10 and len(v.kf_start) == nkf + 1
    assert set(starts.tolist()) <= set(v.kf_start[:-1].tolist())
    assert v.palpix.shape == (10 * tm_w * tm_h, 64) and int(v.dith_pal.max()) < 4
    canon, hm, vm = synth.prepare_tile_mirrors(v.palpix)   # already canonical: no further flip
    assert np.array_equal(canon.reshape(v.palpix.shape), v.palpix) and not hm.any() and not vm.any()
    kf_of = np.repeat(np.arange(nkf), np.diff(v.kf_start))
    px, thm, tvm = oracle.dither_tiles_tk(frames.reshape(-1, 64), (np.repeat(kf_of, tm_w * tm_h) * 4 + v.dith_pal),
                                          pals.reshape(-1, 16))
    assert np.array_equal(px, v.palpix) and np.array_equal(thm, v.thm) and np.array_equal(tvm, v.tvm)


# ---- the Yliluoma branch (chkUseTK unchecked): DeviseBestMixingPlanYliluoma main.pas:1573-1826, ASM_DBMP form ----

def _qs(a, first, last, luma):
    """kmodes.pas:89-136 QuickSort with PlanCompareLuma, in Python (restated again, apart from _py_plan's)."""
    if last <= first:
        return
    while True:
        i, j, p = first, last, (first + last) >> 1
        while True:
            while luma[a[i]] < luma[a[p]]:
                i += 1
            while luma[a[j]] > luma[a[p]]:
                j -= 1
            if i <= j:
                a[i], a[j] = a[j], a[i]
                if p == i:
                    p = j
                elif p == j:
                    p = i
                i += 1
                j -= 1
            if i > j:
                break
        if first < j:
            _qs(a, first, j, luma)
        first = i
        if i >= last:
            break


def _py_yl_plan(pal, col, mixed):
    """The SSE block of main.pas:1602-1752 lane by lane in Python ints: per t, sum += add and add += 1 in all four
    lanes (r, g, b, luma), q = (gVecInv[t] * sum) & 0xffffffff >> 16, pen = sum_k w_k (q_k - x_k)^2 mod 2^32
    (pmulld / psrld / psubd / phaddd), strict '<'; amount = t - plan_count capped by the 256-entry list."""
    M = 0xFFFFFFFF
    rgb = [(c & 255, (c >> 8) & 255, (c >> 16) & 255) for c in pal]
    luma = [r * 2126 + g * 7152 + b * 722 for r, g, b in rgb]
    y2 = [(r, g, b, lu // 10000) for (r, g, b), lu in zip(rgb, luma)]
    r, g, b = col & 255, (col >> 8) & 255, (col >> 16) & 255
    x = (r, g, b, (r * 2126 + g * 7152 + b * 722) // 10000)
    w = (13, 13, 13, 32)
    so, lst, pc = [0, 0, 0, 0], [], 0
    while pc < mixed:
        mt = 1 if pc == 0 else pc
        least, chosen, ct = (1 << 63) - 1, 0, pc + 1
        for idx, yv in enumerate(y2):
            s, a = list(so), list(yv)
            for t in range(pc + 1, pc + mt + 1):
                inv = 65536 // t
                pen = 0
                for k in range(4):
                    s[k] = (s[k] + a[k]) & M
                    a[k] = (a[k] + 1) & M
                    q = ((inv * s[k]) & M) >> 16
                    d = (q - x[k]) & M
                    pen = (pen + (((d * d) & M) * w[k] & M)) & M
                if pen < least:
                    least, chosen, ct = pen, idx, t
        amount = min(ct - pc, 256 - pc)
        lst += [chosen] * amount
        pc += amount
        so = [(so[k] + y2[chosen][k] * amount) & M for k in range(4)]
    _qs(lst, 0, pc - 1, luma)
    return np.asarray(lst, np.uint8), luma


@pytest.mark.parametrize("mixed", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("ties", [False, True])
def test_yl_plan_matches_python(oracle, mixed, ties):
    rng = np.random.default_rng(31 + mixed + 100 * ties)
    for _ in range(3):
        pal = _palette(rng, ties=ties)
        for col in synth.rgb_pack(*rng.integers(0, 256, (3, 12))):
            o = oracle.yl_plan(pal, int(col), mixed)
            p, luma = _py_yl_plan([int(c) for c in pal], int(col), mixed)
            assert np.array_equal(o, p)
            assert mixed <= o.size <= max(1, 2 * (mixed - 1))
            assert all(luma[a] <= luma[b] for a, b in zip(o[:-1], o[1:]))   # sorted by luma


def test_yl_plan_known_answers(oracle):
    pal = _palette(np.random.default_rng(5))
    for i in (0, 9, 15):
        lst = oracle.yl_plan(pal, int(pal[i]), 4)
        assert np.all(lst == i) and lst.size >= 4   # an exact palette colour: mixing it with itself wins
    gray = synth.rgb_pack(*([np.arange(16) * 17] * 3)).astype(np.int32)
    lst = oracle.yl_plan(gray, int(synth.rgb_pack(25, 25, 25)), 8)  # between entries 1 (17) and 2 (34)
    assert set(lst.tolist()) <= {1, 2}


def test_dither_tiles_yl_composition(oracle):
    """or_dither_tiles_yl = per-pixel plan -> list[cDitheringMap * count shr 6] -> PrepareTileMirrors."""
    rng = np.random.default_rng(9)
    pals = np.stack([_palette(rng, ties=k % 2 == 1) for k in range(3)])
    rgb = synth.frame_tiles(rng, 6)
    pal_of = rng.integers(0, 3, 6).astype(np.int32)
    px, hm, vm = oracle.dither_tiles_yl(rgb, pal_of, pals, 4)
    raw = np.zeros((6, 64), np.uint8)
    for t in range(6):
        for k in range(64):
            lst = oracle.yl_plan(pals[pal_of[t]], int(rgb[t, k]), 4)
            raw[t, k] = lst[(MAP[k] * lst.size) >> 6]
    cpx, chm, cvm = synth.prepare_tile_mirrors(raw)
    assert np.array_equal(px, cpx.reshape(6, 64)) and np.array_equal(hm, chm) and np.array_equal(vm, cvm)

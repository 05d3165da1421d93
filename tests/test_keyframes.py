"""Load-step keyframe detection (btnLoadClick main.pas:1099-1146): the CPU restatement
(oracle/load_kf.c) against known answers and an independent pure-Python evaluation, and the shot split
(host code of libANN.so, tiler_find_keyframes) against the restatement.  No reference fixture exists for
this step (no FPC, no frames in the reference): parity against the reference binary is unpinned; the
evaluation order is restated from main.pas:811-828 and 1465-1492."""
import math

import numpy as np
import pytest

from tiler_amd import synth
from tiler_amd.keyframes import find_keyframes, keyframe_starts


def _py_pearson(a, b, tm_w, tm_h):
    """Independent restatement: build ya/yb exactly as ComputeInterFrameCorrelation (main.pas:811-828) does
    (FSPixels in raster order, planar copy), then PearsonCorrelation (main.pas:1465-1492) in Python floats."""
    def fs(t):
        img = np.asarray(t).reshape(tm_h, tm_w, 8, 8).transpose(0, 2, 1, 3).reshape(-1)
        px = np.stack([img & 255, (img >> 8) & 255, (img >> 16) & 255], 1).reshape(-1)  # FSPixels r,g,b
        sz = px.size // 3
        return [float(px[i * 3 + c]) for c in range(3) for i in range(sz)]
    x, y = fs(a), fs(b)
    mx, my = sum(x) / len(x), sum(y) / len(y)
    num = denx = deny = 0.0
    for xi, yi in zip(x, y):
        num += (xi - mx) * (yi - my)
        denx += (xi - mx) * (xi - mx)
        deny += (yi - my) * (yi - my)
    den = math.sqrt(denx) * math.sqrt(deny)
    return num / den if den != 0.0 else 0.0


def _py_split(corr, F, tms):
    """main.pas:1099-1132 in Python."""
    kf, last, av, out = 0, 0, -1.0, [0] * F
    for i in range(1, F):
        v = corr[i - 1]
        av = v if av == -1.0 else av * (1.0 - 1.0 / 6) + v * (1.0 / 6)
        ratio = max(0.01, v) / max(0.01, av)
        if ratio < 0.5 or (ratio < 0.9 and (i - last + 1) > 24) or (i - last + 1) * tms > 24 * 1920 * 1080 // 64:
            kf, av, last = kf + 1, -1.0, i
        out[i] = kf
    return np.asarray(out, np.int32), kf + 1


def test_pearson_matches_python_restatement_bit_exact(oracle):
    rng = np.random.default_rng(5)
    frames, _ = synth.shot_frames(rng, 6, 3, 2, shot_len=(2, 3))
    corr = oracle.interframe_corr_batch(frames, 3, 2)
    for i in range(1, 6):
        assert corr[i - 1] == _py_pearson(frames[i - 1], frames[i], 3, 2)


def test_pearson_known_answers(oracle):
    rng = np.random.default_rng(6)
    a = synth.rgb_pack(*rng.integers(0, 256, (3, 4, 64)))
    flat = np.full((4, 64), synth.rgb_pack(77, 77, 77), np.int32)  # constant planar array
    inv = synth.rgb_pack(255 - (a & 255), 255 - ((a >> 8) & 255), 255 - ((a >> 16) & 255))
    c = oracle.interframe_corr_batch(np.stack([a, a, flat, a, inv]), 2, 2)
    assert abs(c[0] - 1.0) < 1e-15          # identical frames
    assert c[1] == 0.0 and c[2] == 0.0      # den = 0 -> Result := 0.0 (main.pas:1489-1491)
    assert abs(c[3] + 1.0) < 1e-15          # negated bytes
    ref = np.corrcoef(*[np.stack([(f >> (8 * k)) & 255 for k in range(3)]).reshape(-1) for f in (a, inv)])[0, 1]
    assert abs(c[3] - ref) < 1e-12


def test_pearson_close_to_numpy_on_shots(oracle):
    rng = np.random.default_rng(7)
    frames, _ = synth.shot_frames(rng, 12, 10, 6, shot_len=(3, 6))
    corr = oracle.interframe_corr_batch(frames, 10, 6)
    for i in range(1, 12):
        x, y = [np.stack([(frames[j] >> (8 * k)) & 255 for k in range(3)]).reshape(-1) for j in (i - 1, i)]
        assert abs(corr[i - 1] - np.corrcoef(x, y)[0, 1]) < 1e-12


@pytest.mark.parametrize("case", ["hard", "soft_grace", "span_cap", "random"])
def test_split_matches_restatement(oracle, case):
    rng = np.random.default_rng(hash(case) % 2**32)
    F, tms = 200, 40 * 30
    if case == "hard":
        corr = np.full(F - 1, 0.95)
        corr[[10, 50, 51, 120]] = [0.3, 0.2, 0.9, 0.4]
    elif case == "soft_grace":      # ratio in [0.5, 0.9): a cut only after the 24-frame grace period
        corr = np.full(F - 1, 0.9)
        corr[[5, 40, 41, 90]] = 0.7
    elif case == "span_cap":        # 1080p: at most 24 frames per keyframe (CShotTransMaxTilesPerKF)
        corr, tms = np.full(F - 1, 0.99), 240 * 135
    else:
        corr = np.clip(rng.normal(0.85, 0.2, F - 1), -1, 1)
    kf, n = find_keyframes(corr, F, tms)     # libANN.so host code
    okf, on = oracle.find_keyframes(corr, F, tms)
    pkf, pn = _py_split(corr, F, tms)
    assert n == on == pn and np.array_equal(kf, okf) and np.array_equal(kf, pkf)
    if case == "hard":
        assert set(np.flatnonzero(np.diff(kf)) + 1) == {11, 51, 121}
    if case == "soft_grace":
        assert set(np.flatnonzero(np.diff(kf)) + 1) == {41, 91}
    if case == "span_cap":
        assert np.all(np.diff(keyframe_starts(kf))[:-1] == 24)


def test_split_edges(oracle):
    assert find_keyframes(np.zeros(0), 0, 100)[1] == 0
    kf, n = find_keyframes(np.zeros(0), 1, 100)
    assert n == 1 and list(kf) == [0]
    assert list(keyframe_starts([0, 0, 1, 1, 1, 2])) == [0, 2, 5, 6]

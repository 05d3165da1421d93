"""GPU parity of the Load step's keyframe detection (ComputeInterFrameCorrelation main.pas:811-828 +
btnLoadClick's split main.pas:1099-1146): correlations bit-identical to the sequential fp64 restatement,
keyframe indices equal."""
import numpy as np
import pytest

from tiler_amd import synth
from tiler_amd.keyframes import detect_keyframes, interframe_correlation

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("F,tm_w,tm_h", [(0, 4, 3), (1, 4, 3), (2, 4, 3), (70, 20, 12), (130, 7, 5)])
def test_correlation_bit_exact(gpu, oracle, F, tm_w, tm_h):
    """Ragged frame counts around the 64-frame wave (one lane per frame) and odd tilemap sizes."""
    rng = np.random.default_rng(F * 131 + tm_w)
    frames, _ = synth.shot_frames(rng, max(F, 1), tm_w, tm_h, shot_len=(3, 30))
    frames = frames[:F]
    g = interframe_correlation(frames, tm_w, tm_h)
    o = oracle.interframe_corr_batch(frames, tm_w, tm_h)
    assert g.shape == o.shape == (max(0, F - 1),)
    assert np.array_equal(g.view(np.uint64), o.view(np.uint64))


def test_correlation_edge_frames(gpu, oracle):
    """Constant frames (den = 0 -> 0.0), identical and negated neighbours."""
    rng = np.random.default_rng(3)
    a = synth.rgb_pack(*rng.integers(0, 256, (3, 12, 64)))
    flat = np.full_like(a, synth.rgb_pack(77, 77, 77))
    inv = synth.rgb_pack(255 - (a & 255), 255 - ((a >> 8) & 255), 255 - ((a >> 16) & 255))
    frames = np.stack([a, a, flat, flat, a, inv, np.zeros_like(a)])
    g = interframe_correlation(frames, 4, 3)
    o = oracle.interframe_corr_batch(frames, 4, 3)
    assert np.array_equal(g.view(np.uint64), o.view(np.uint64))
    assert g[2] == 0.0 and g[5] == 0.0


def test_1080p_clip_keyframes(gpu, oracle):
    """Full 1080p frames (240x135 tiles, the reference's cap): correlations bit-exact and the same keyframes
    as the restatement; every synthetic shot cut is found.  (The HBM-resident entry point,
    tiler_interframe_correlation_dev, is what the host entry runs after its copy; bench.py calls it directly
    on torch-allocated frames and re-checks the result bit for bit.)"""
    rng = np.random.default_rng(11)
    F, tm_w, tm_h = 40, 240, 135
    frames, starts = synth.shot_frames(rng, F, tm_w, tm_h, shot_len=(5, 14))
    g = interframe_correlation(frames, tm_w, tm_h)
    o = oracle.interframe_corr_batch(frames, tm_w, tm_h)
    assert np.array_equal(g.view(np.uint64), o.view(np.uint64))
    kf, kf_start, corr = detect_keyframes(frames, tm_w, tm_h)
    okf, _ = oracle.find_keyframes(o, F, tm_w * tm_h)
    assert np.array_equal(kf, okf)
    assert set(starts.tolist()) <= set(kf_start[:-1].tolist())


def test_4k_frames_beyond_reference_cap(gpu, oracle):
    """4K frames (480x270 tiles, past ReframeUI's 1080p cap main.pas:1933-1934, as C5 uses them): bit-exact."""
    rng = np.random.default_rng(13)
    frames, _ = synth.shot_frames(rng, 3, 480, 270, shot_len=(2, 2))
    g = interframe_correlation(frames, 480, 270)
    o = oracle.interframe_corr_batch(frames, 480, 270)
    assert np.array_equal(g.view(np.uint64), o.view(np.uint64))

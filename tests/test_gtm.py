"""GTM writer + LZMA: SaveStream (main.pas:4529-4763) and LZCompress (extern.pas:202-240).

Pins: the oracle's LZMA-alone decoder (oracle/lzma_dec.c) reads the reference's own demo streams
(docs/demo/*.gtm, written by the reference encoder through lzma.exe -lc8; committed facts in
tests/golden/gtm_demo.json), so it checks libANN.so's encoder; the GTM reader follows the reference
player's command semantics (tests/gtm_read.py).  All CPU: the encoder is host code."""
import hashlib
import json
import os

import numpy as np
import pytest

from gtm_read import lzma_decode_all, read_gtm, render
from tiler_amd import gtm

HERE = os.path.dirname(os.path.abspath(__file__))
DEMO = "/root/reference/docs/demo"


def _roundtrip(oracle, data: bytes, **kw):
    comp = gtm.lzma_encode(data, **kw)
    outs, end = lzma_decode_all(oracle, comp, 0)
    assert end == len(comp) and len(outs) == 1
    return comp, outs[0]


@pytest.mark.parametrize("props", [(8, 0, 2), (3, 0, 2), (0, 4, 0), (4, 2, 4), (8, 4, 4)])
def test_lzma_roundtrip(oracle, props):
    lc, lp, pb = props
    rng = np.random.default_rng(lc * 25 + lp * 5 + pb)
    cases = [b"", b"\x07", bytes(100000), rng.integers(0, 256, 30000, dtype=np.uint8).tobytes(),
             rng.integers(0, 4, 100000, dtype=np.uint8).tobytes(),
             np.tile(rng.integers(0, 256, 777, dtype=np.uint8), 200).tobytes(),
             open(os.path.join(HERE, "..", "DESIGN.md"), "rb").read()]
    for data in cases:
        comp, back = _roundtrip(oracle, data, lc=lc, lp=lp, pb=pb)
        assert back == data
        assert comp[0] == (pb * 5 + lp) * 9 + lc and comp[5:13] == b"\xff" * 8
    # known-size header (no end marker)
    comp, back = _roundtrip(oracle, cases[5], eos=False)
    assert back == cases[5] and int.from_bytes(comp[5:13], "little") == len(cases[5])


def test_lzma_bad_args():
    with pytest.raises(RuntimeError):
        gtm.lzma_encode(b"abc", lc=9)


@pytest.mark.skipif(not os.path.isdir(DEMO), reason="reference demo streams not present")
def test_reference_demo_streams(oracle):
    """The reference's own .gtm demos decode completely (every frame's tilemap full, indices in range) and
    match the committed facts; re-encoding their raw streams with libANN.so's encoder round-trips."""
    golden = json.load(open(os.path.join(HERE, "golden", "gtm_demo.json")))
    for name, want in golden.items():
        data = open(os.path.join(DEMO, name), "rb").read()
        assert hashlib.sha256(data).hexdigest() == want["file_sha256"]
        g = read_gtm(oracle, data)
        assert [len(s) for s in g.streams] == want["streams_raw_bytes"]
        assert [hashlib.sha256(s).hexdigest() for s in g.streams] == want["streams_sha256"]
        assert (g.width, g.height, g.frame_ns, g.tiles.shape[0], len(g.frames)) == \
            (want["width"], want["height"], want["frame_ns"], want["tiles"], want["frames"])
        assert hashlib.sha256(render(g).tobytes()).hexdigest() == want["rendered_sha256"]
        assert g.stream_comp == want["streams_compressed_bytes"]
        s, ref_len = g.streams[-1], g.stream_comp[-1]  # the smaller stream keeps the CPU suite quick
        comp, back = _roundtrip(oracle, s)
        assert back == s and len(comp) < 1.15 * ref_len  # vs the reference's lzma.exe on the same bytes


def _smoothed_maps(rng, F, Q, T, P):
    tile = rng.integers(0, T, (F, Q))
    pal = rng.integers(0, P, (F, Q))
    hm = rng.integers(0, 2, (F, Q)).astype(np.uint8)
    vm = rng.integers(0, 2, (F, Q)).astype(np.uint8)
    sm = np.zeros((F, Q), np.uint8)
    for f in range(1, F):
        keep = rng.random(Q) < 0.6
        s0 = int(rng.integers(0, Q - 1100))
        keep[s0:s0 + 1100] = True  # a run longer than the 1024-item skip limit
        tile[f] = np.where(keep, tile[f - 1], tile[f])
        pal[f] = np.where(keep, pal[f - 1], pal[f])
        hm[f] = np.where(keep, hm[f - 1], hm[f])
        vm[f] = np.where(keep, vm[f - 1], vm[f])
        sm[f] = keep
    return tile, pal, hm, vm, sm


@pytest.mark.parametrize("T", [300, 70000])
def test_save_stream_roundtrip(oracle, T):
    """SaveStream -> reader: header / keyframe records per main.pas:4632-4757, tiles, palettes, and every
    frame's items (skips exactly at the Smoothed items, Short/LongTileIdx by index size, mirrors xored with
    the tile's canonical flags); the rendered frames equal a direct rendering of the SmoothedTileMaps."""
    rng = np.random.default_rng(T)
    W, H, P, fps = 320, 240, 6, 30.0
    Q = (W // 8) * (H // 8)
    kf_start = np.array([0, 3, 4, 8])
    F = int(kf_start[-1])
    palpix = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    thm = rng.integers(0, 2, T).astype(np.uint8)
    tvm = rng.integers(0, 2, T).astype(np.uint8)
    pals = rng.integers(0, 1 << 24, (3, P, 16)).astype(np.int32)
    tile, pal, hm, vm, sm = _smoothed_maps(rng, F, Q, T, P)
    for k in range(3):
        sm[kf_start[k]] = 0  # the first frame of a keyframe is never smoothed (main.pas:4081-4082)
    data = gtm.save_stream(palpix, thm, tvm, kf_start, pals, tile, pal, hm, vm, sm, W, H, fps)
    g = read_gtm(oracle, data)
    h = g.header
    assert (h["RIFFSize"], h["WholeHeaderSize"], h["EncoderVersion"], h["FramePixelWidth"], h["FramePixelHeight"],
            h["KFCount"], h["FrameCount"]) == (32, 40 + 28 * 3, 1, W, H, 3, F)
    comp = [k["CompressedSize"] for k in g.kfinfo]
    assert sum(comp) == len(data) - h["WholeHeaderSize"] and [len(s) > 0 for s in g.streams] == [True] * 3
    assert [k["FrameIndex"] for k in g.kfinfo] == [0, 3, 4]
    assert [k["TimeCodeMillisecond"] for k in g.kfinfo] == [0, 100, 133]
    assert h["AverageBytesPerSec"] == round(sum(comp) * fps / F)
    assert h["KFMaxBytesPerSec"] == max(round(comp[1] * fps / 1), round(comp[2] * fps / 4))
    assert (g.width, g.height, g.frame_ns, g.palsize) == (W // 8, H // 8, 33333333, 16)
    assert np.array_equal(g.tiles, palpix)
    assert [f[2] for f in g.frames] == [0, 0, 1, 1, 0, 0, 0, 1]
    expect = np.zeros((H, W, 4), np.uint8)
    for f, (items, pl, _) in enumerate(g.frames):
        k = int(np.searchsorted(kf_start, f, side="right") - 1)
        for j in range(P):
            rgba = np.ascontiguousarray(pl[j]).view(np.uint32).ravel()
            assert np.array_equal(rgba, pals[k, j].astype(np.uint32) | 0xFF000000)
        skipped = items[:, 0] < 0
        assert np.array_equal(skipped, sm[f].astype(bool))
        live = ~skipped
        assert np.array_equal(items[live, 0], tile[f][live])
        attrs = (pal[f] << 2) | ((vm[f] ^ tvm[tile[f]]) << 1) | (hm[f] ^ thm[tile[f]])
        assert np.array_equal(items[live, 1], attrs[live])
    # render the intended display directly: tile flipped by (item mirror xor canonical), palette colours
    fr = render(g)
    for f in range(F):
        k = int(np.searchsorted(kf_start, f, side="right") - 1)
        for q in np.nonzero(~sm[f].astype(bool))[0]:
            t = palpix[tile[f, q]].reshape(8, 8)
            if hm[f, q] ^ thm[tile[f, q]]:
                t = t[:, ::-1]
            if vm[f, q] ^ tvm[tile[f, q]]:
                t = t[::-1, :]
            col = (pals[k, pal[f, q]].astype(np.uint32) | 0xFF000000).view(np.uint8).reshape(16, 4)
            y, x = divmod(int(q), W // 8)
            expect[y * 8:y * 8 + 8, x * 8:x * 8 + 8] = col[t]
        assert np.array_equal(fr[f], expect)

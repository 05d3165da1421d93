"""TEST INFRASTRUCTURE: a GTM reader (the command semantics of the reference player,
decoders/htmljs/gtm.player.js:257-345) over the oracle's LZMA-alone decoder (oracle/lzma_dec.c), and an
RGBA renderer with the player's tile drawing (drawTilemapItem, gtm.player.js:171-241)."""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass, field

import numpy as np


def lzma_decode_all(oracle, data: bytes, start: int, comp_sizes: list | None = None):
    """Decode the concatenated LZMA-alone streams from `start`; returns (list of raw streams, end offset).
    `comp_sizes`, if given, receives each stream's compressed size."""
    f = oracle.lib().or_lzma_decode
    f.restype = ctypes.c_long
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    buf = np.frombuffer(data, np.uint8)
    pos, outs = start, []
    while pos < len(data):
        cap = 1 << 20
        while True:
            out = np.zeros(cap, np.uint8)
            used = ctypes.c_size_t(0)
            seg = np.ascontiguousarray(buf[pos:])
            r = f(seg.ctypes.data_as(ctypes.c_void_p), seg.size, out.ctypes.data_as(ctypes.c_void_p), cap,
                  ctypes.byref(used))
            if r == -2:
                cap *= 4
                continue
            if r < 0:
                raise ValueError(f"corrupt LZMA stream at {pos}")
            break
        outs.append(out[:r].tobytes())
        pos += used.value
        if comp_sizes is not None:
            comp_sizes.append(used.value)
    return outs, pos


@dataclass
class GTM:
    header: dict
    kfinfo: list
    width: int = 0
    height: int = 0
    frame_ns: int = 0
    tiles: np.ndarray = None
    palsize: int = 0
    streams: list = field(default_factory=list)
    stream_comp: list = field(default_factory=list)  # compressed bytes per stream
    # per frame: items [Q] (tile, attrs) with -1 tile where skipped; palettes at that frame
    frames: list = field(default_factory=list)


def read_gtm(oracle, data: bytes) -> GTM:
    names = ["FourCC", "RIFFSize", "WholeHeaderSize", "EncoderVersion", "FramePixelWidth", "FramePixelHeight",
             "KFCount", "FrameCount", "AverageBytesPerSec", "KFMaxBytesPerSec"]
    kfi = []
    if data[:4] != b"GTMv":  # headerless stream (the player's parseHeader fallback, gtm.player.js:137-139)
        g = GTM({}, [])
        hdr = {"WholeHeaderSize": 0, "KFCount": 0}
    else:
        hdr = dict(zip(names, struct.unpack_from("<10I", data, 0)))
    for k in range(hdr["KFCount"]):
        v = struct.unpack_from("<7I", data, 40 + 28 * k)
        assert data[40 + 28 * k:44 + 28 * k] == b"GTMk"
        kfi.append(dict(zip(["FourCC", "RIFFSize", "KFIndex", "FrameIndex", "RawSize", "CompressedSize",
                             "TimeCodeMillisecond"], v)))
    g = GTM(hdr, kfi)
    g.streams, _ = lzma_decode_all(oracle, data, hdr["WholeHeaderSize"], g.stream_comp)
    raw = b"".join(g.streams)
    pos = 0
    pal = {}
    cur = None

    def rd(fmt):
        nonlocal pos
        v = struct.unpack_from(fmt, raw, pos)
        pos += struct.calcsize(fmt)
        return v[0] if len(v) == 1 else v

    tm = 0
    while pos < len(raw):
        w = rd("<H")
        cmd, arg = w & 63, w >> 6
        if cmd == 30:  # SetDimensions
            g.width, g.height, g.frame_ns, count = rd("<HHII")
            g.tiles = np.zeros((count, 64), np.uint8)
            cur = np.full((g.width * g.height, 2), -1, np.int64)
        elif cmd == 29:  # TileSet
            t0, t1 = rd("<II")
            g.palsize = arg
            n = t1 - t0 + 1
            g.tiles[t0:t1 + 1] = np.frombuffer(raw, np.uint8, n * 64, pos).reshape(n, 64)
            pos += n * 64
        elif cmd == 3:  # LoadPalette
            idx, _fmt = rd("<BB")
            pal[idx] = np.frombuffer(raw, np.uint8, 4 * g.palsize, pos).reshape(g.palsize, 4).copy()
            pos += 4 * g.palsize
        elif cmd == 0:  # SkipBlock
            tm += arg + 1
        elif cmd in (1, 2):
            t = rd("<H") if cmd == 1 else rd("<I")
            cur[tm] = (t, arg)
            tm += 1
        elif cmd == 28:  # FrameEnd
            assert tm == g.width * g.height, (tm, g.width * g.height)
            g.frames.append((cur.copy(), {k: v.copy() for k, v in pal.items()}, arg & 1))
            cur[:] = -1
            tm = 0
        else:
            raise ValueError(f"unknown GTM command {cmd}")
    return g


def render(g: GTM):
    """RGBA frames [F][H*8][W*8][4] as the player draws them (skips keep the previous pixels)."""
    H, W = g.height, g.width
    img = np.zeros((H * 8, W * 8, 4), np.uint8)
    out = []
    for items, pal, _ in g.frames:
        for yx in np.nonzero(items[:, 0] >= 0)[0]:
            t, attrs = items[yx]
            tile = g.tiles[t].reshape(8, 8)
            if attrs & 1:
                tile = tile[:, ::-1]
            if attrs & 2:
                tile = tile[::-1, :]
            y, x = divmod(int(yx), W)
            img[y * 8:y * 8 + 8, x * 8:x * 8 + 8] = pal[int(attrs) >> 2][tile]
        out.append(img.copy())
    return np.stack(out) if out else np.zeros((0, H * 8, W * 8, 4), np.uint8)

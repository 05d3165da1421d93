"""GTM bitstream writer (SaveStream main.pas:4529-4763) over libANN.so's LZMA-alone encoder.

`save_stream` follows the reference procedure step by step:
  header        TGTMHeader (main.pas:103-114) + one TGTMKeyFrameInfo per keyframe (116-124), rewritten at
                the end with the measured sizes (4753-4757);
  per keyframe  one LZMA-alone stream (LZCompress extern.pas:202-240: `lzma.exe e -lc8 -eos` ->
                tiler_lzma_encode(lc=8, lp=0, pb=2, eos)) of the command words (DoCmd 4565-4571: data << 6 | cmd):
                  first keyframe only: WriteTiles (4603-4622) = SetDimensions + TileSet + 64 B per tile,
                  WriteKFAttributes (4589-4601) = LoadPalette per palette,
                  per frame the SmoothedTileMap: runs of Smoothed items -> SkipBlock (count - 1, at most
                  2^10), others -> Short/LongTileIdx with (PalIdx << 2 | VMirror' << 1 | HMirror'), where the
                  mirrors are xored with the tile's canonical flags (4715), then FrameEnd(is last frame of KF).
The reference takes these bytes verbatim from lzma.exe; this build's encoder makes a different (valid)
parse, so the compressed bytes differ while everything a decoder returns is identical.
"""
from __future__ import annotations

import ctypes
import os
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ._lib import check, load

GT_SKIP_BLOCK, GT_SHORT_TILE_IDX, GT_LONG_TILE_IDX, GT_LOAD_PALETTE = 0, 1, 2, 3
GT_FRAME_END, GT_TILE_SET, GT_SET_DIMENSIONS = 28, 29, 30
CMD_BITS = 6                      # round(ln(64) / ln(2)), main.pas:4532
ATTR_BITS = 16 - CMD_BITS         # 10
MAX_BLK_SKIP = 1 << ATTR_BITS     # CMaxBlkSkipCount main.pas:4535
LZMA_LC, LZMA_LP, LZMA_PB = 8, 0, 2
LZMA_DICT = 1 << 21             # the reference's lzma.exe streams (docs/demo/*.gtm headers)


def lzma_encode(data: bytes, lc: int = LZMA_LC, lp: int = LZMA_LP, pb: int = LZMA_PB, dict_size: int = LZMA_DICT,
                eos: bool = True) -> bytes:
    """LZCompress (extern.pas:202-240) on libANN.so: one LZMA-alone stream."""
    lib = load()
    src = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
    n = ctypes.c_size_t(0)
    p = src.ctypes.data_as(ctypes.c_void_p)
    out = np.zeros(len(data) + len(data) // 32 + 4096, np.uint8)  # LZMA expands incompressible data < 2 %
    if lib.tiler_lzma_encode(p, len(data), lc, lp, pb, dict_size, int(eos), out.ctypes.data_as(ctypes.c_void_p),
                             out.size, ctypes.byref(n)) != 0:
        out = np.zeros(n.value, np.uint8)
        check(lib.tiler_lzma_encode(p, len(data), lc, lp, pb, dict_size, int(eos),
                                    out.ctypes.data_as(ctypes.c_void_p), out.size, ctypes.byref(n)),
              "tiler_lzma_encode")
    return out[:n.value].tobytes()


def fpc_round(x: float) -> int:
    """FPC Round: banker's rounding (Python's round)."""
    return int(round(x))


class _Z:
    def __init__(self):
        self.b = bytearray()

    def cmd(self, c: int, data: int):
        assert 0 <= data < (1 << ATTR_BITS) and 0 <= c < 64
        self.b += struct.pack("<H", (data << CMD_BITS) | c)

    def word(self, v):
        self.b += struct.pack("<H", v)

    def dword(self, v):
        self.b += struct.pack("<I", v & 0xFFFFFFFF)

    def byte(self, v):
        self.b.append(v & 0xFF)


def _frame_words(tile, pal, hm, vm, smb, thm, tvm, is_last: bool) -> np.ndarray:
    """One frame's command words in position order (main.pas:4675-4725), vectorised: every run of Smoothed
    items becomes SkipBlock words of at most 2^10 items, every other item Short/LongTileIdx + its index."""
    d = np.diff(np.concatenate([[0], smb.astype(np.int8), [0]]))
    starts, ends = np.nonzero(d == 1)[0], np.nonzero(d == -1)[0]
    nch = (ends - starts + MAX_BLK_SKIP - 1) // MAX_BLK_SKIP
    first = np.repeat(np.cumsum(nch) - nch, nch)
    cstart = np.repeat(starts, nch) + MAX_BLK_SKIP * (np.arange(int(nch.sum())) - first)
    clen = np.minimum(MAX_BLK_SKIP, np.repeat(ends, nch) - cstart)
    live = np.nonzero(~smb)[0]
    t = tile[live]
    attrs = (pal[live] << 2) | ((vm[live] ^ tvm[t]) << 1) | (hm[live] ^ thm[t])
    assert (attrs < (1 << ATTR_BITS)).all() and (pal >= 0).all()
    long_ = t >= (1 << 16)
    nc = cstart.size
    words = np.zeros((nc + live.size, 3), np.uint16)
    words[:nc, 0] = ((clen - 1) << CMD_BITS) | GT_SKIP_BLOCK
    words[nc:, 0] = (attrs << CMD_BITS) | np.where(long_, GT_LONG_TILE_IDX, GT_SHORT_TILE_IDX)
    words[nc:, 1] = t & 0xFFFF
    words[nc:, 2] = t >> 16
    nwords = np.concatenate([np.ones(nc, np.int64), np.where(long_, 3, 2)])
    order = np.argsort(np.concatenate([cstart, live]), kind="stable")
    words, nwords = words[order], nwords[order]
    out = words[np.arange(3)[None, :] < nwords[:, None]]  # row-major: each token's words in order
    end = np.array([(int(is_last) << CMD_BITS) | GT_FRAME_END], np.uint16)
    return np.concatenate([out, end]).astype("<u2")


def keyframe_commands(tile, pal, hm, vm, smoothed, thm, tvm, palettes, palsize: int = 16):
    """The command words of one keyframe's frames ([F][Q] SmoothedTileMap arrays), after WriteKFAttributes."""
    z = _Z()
    for j in range(palettes.shape[0]):  # WriteKFAttributes
        z.cmd(GT_LOAD_PALETTE, 0)
        z.byte(j)
        z.byte(0)
        for i in range(palsize):
            z.dword(int(palettes[j, i]) | 0xFF000000)
    F, Q = tile.shape
    thm = np.asarray(thm, np.int64)
    tvm = np.asarray(tvm, np.int64)
    for f in range(F):
        z.b += _frame_words(np.asarray(tile[f], np.int64), np.asarray(pal[f], np.int64), np.asarray(hm[f], np.int64),
                            np.asarray(vm[f], np.int64), np.asarray(smoothed[f]).astype(bool), thm, tvm,
                            f == F - 1).tobytes()
    return bytes(z.b)


def keyframe_raw(k: int, palpix, thm, tvm, palettes_k, tile, pal, hm, vm, smoothed, *, width: int, height: int,
                 fps: float, palsize: int = 16) -> bytes:
    """The uncompressed command bytes of keyframe k (SaveStream main.pas:4724-4734): WriteTiles for k = 0 only
    (SetDimensions + TileSet + 64 B per tile, 4603-4622), then WriteKFAttributes and the keyframe's frames
    (tile/pal/hm/vm/smoothed: its [f][Q] SmoothedTileMap rows)."""
    palpix = np.ascontiguousarray(palpix, np.uint8).reshape(-1, 64)
    T = palpix.shape[0]
    z = _Z()
    if k == 0:  # WriteTiles
        z.cmd(GT_SET_DIMENSIONS, 0)
        z.word(width // 8)
        z.word(height // 8)
        z.dword(fpc_round(1000 * 1000 * 1000 / fps))
        z.dword(T)
        z.cmd(GT_TILE_SET, palsize)
        z.dword(0)
        z.dword(T - 1)
        z.b += palpix.tobytes()
    z.b += keyframe_commands(tile, pal, hm, vm, smoothed, thm, tvm, palettes_k, palsize)
    return bytes(z.b)


def compress_streams(raws, threads: int | None = None) -> list:
    """LZCompress of independent keyframe streams, concurrently (the C encoder runs outside the GIL)."""
    if not raws:
        return []
    workers = max(1, min(len(raws), threads or min(16, len(os.sched_getaffinity(0)))))
    with ThreadPoolExecutor(workers) as ex:
        return list(ex.map(lzma_encode, raws))


def assemble_stream(comps, kf_start, width: int, height: int, fps: float) -> bytes:
    """The .gtm file from the keyframes' compressed streams (in keyframe order): TGTMHeader (main.pas:103-114),
    one TGTMKeyFrameInfo per keyframe (116-124) with the measured sizes (4735-4757), then the streams."""
    kf_start = np.asarray(kf_start, np.int64)
    KF = kf_start.size - 1
    F = int(kf_start[-1])
    header = {"AverageBytesPerSec": 0, "KFMaxBytesPerSec": 0}
    kfinfo = []
    for k in range(KF):
        kfinfo.append({"KFIndex": k, "FrameIndex": int(kf_start[k]), "RawSize": 0, "CompressedSize": 0,
                       "TimeCodeMillisecond": fpc_round(1000.0 * int(kf_start[k]) / fps)})
    body = bytearray()
    avg = 0
    last_kf = 0
    for k, comp in enumerate(comps):
        f1 = int(kf_start[k + 1])
        body += comp
        kf_count = (f1 - 1) - last_kf + 1
        last_kf = f1
        kfinfo[k]["RawSize"] = 0  # the reference reads ZStream.Size after ZStream.Clear (main.pas:4735-4739)
        kfinfo[k]["CompressedSize"] = len(comp)
        if k > 0 or KF == 1:
            header["KFMaxBytesPerSec"] = max(header["KFMaxBytesPerSec"], fpc_round(len(comp) * fps / kf_count))
        avg += len(comp)
    header["AverageBytesPerSec"] = fpc_round(avg * fps / F)
    h = b"GTMv" + struct.pack("<9I", 40 - 8, 40 + 28 * KF, 1, width, height, KF, F,
                              header["AverageBytesPerSec"] & 0xFFFFFFFF, header["KFMaxBytesPerSec"] & 0xFFFFFFFF)
    for ki in kfinfo:
        h += b"GTMk" + struct.pack("<6I", 28 - 8, ki["KFIndex"], ki["FrameIndex"], ki["RawSize"],
                                   ki["CompressedSize"], ki["TimeCodeMillisecond"])
    return h + bytes(body)


def save_stream(palpix, thm, tvm, kf_start, palettes, sm_tile, sm_pal, sm_hm, sm_vm, sm_smoothed, width: int,
                height: int, fps: float, palsize: int = 16, threads: int | None = None) -> bytes:
    """SaveStream main.pas:4529-4763.  palpix [T][64] (active tiles, reindexed), thm/tvm [T], kf_start [KF+1],
    palettes [KF][P][16], sm_* [F][Q] SmoothedTileMap; width/height in pixels.  Returns the .gtm bytes."""
    kf_start = np.asarray(kf_start, np.int64)
    raws = []
    for k in range(kf_start.size - 1):
        f0, f1 = int(kf_start[k]), int(kf_start[k + 1])
        raws.append(keyframe_raw(k, palpix, thm, tvm, palettes[k], sm_tile[f0:f1], sm_pal[f0:f1], sm_hm[f0:f1],
                                 sm_vm[f0:f1], sm_smoothed[f0:f1], width=width, height=height, fps=fps,
                                 palsize=palsize))
    return assemble_stream(compress_streams(raws, threads), kf_start, width, height, fps)

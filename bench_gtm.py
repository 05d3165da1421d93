"""SaveStream throughput: the GTM writer + per-keyframe LZMA-alone streams (libANN.so's
tiler_lzma_encode, lc=8 lp=0 pb=2, end marker) on a C3-shaped synthetic encode: 1080p (32,400 tiles per
frame), keyframes of 24 frames, a 64k reindexed tileset, SmoothedTileMaps with temporal coherence.  Host
code: the keyframe streams are independent and compressed concurrently.  Prints one JSON line; with
--check the output is read back through the oracle's decoder.

`python bench_gtm.py [--keyframes 8] [--threads 16] [--check]`
"""
from __future__ import annotations

import argparse
import json
import lzma
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tiler_amd import gtm  # noqa: E402


def workload(seed: int, keyframes: int, frames_per_kf: int = 24, W: int = 1920, H: int = 1080, T: int = 65536,
             P: int = 128):
    rng = np.random.default_rng(seed)
    Q = (W // 8) * (H // 8)
    F = keyframes * frames_per_kf
    palpix = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    thm = rng.integers(0, 2, T).astype(np.uint8)
    tvm = rng.integers(0, 2, T).astype(np.uint8)
    pals = rng.integers(0, 1 << 24, (keyframes, P, 16)).astype(np.int32)
    # reindexed tiles: use counts decay with the index (ReindexTiles orders by UseCount)
    w = 1.0 / np.arange(1, T + 1) ** 0.9
    cdf = np.cumsum(w / w.sum())
    tile = np.searchsorted(cdf, rng.random((F, Q))).astype(np.int64)
    pal = rng.integers(0, P, (F, Q))
    hm = rng.integers(0, 2, (F, Q)).astype(np.uint8)
    vm = rng.integers(0, 2, (F, Q)).astype(np.uint8)
    sm = np.zeros((F, Q), np.uint8)
    for f in range(F):
        if f % frames_per_kf == 0:
            continue
        keep = rng.random(Q) < 0.7
        tile[f] = np.where(keep, tile[f - 1], tile[f])
        pal[f] = np.where(keep, pal[f - 1], pal[f])
        hm[f] = np.where(keep, hm[f - 1], hm[f])
        vm[f] = np.where(keep, vm[f - 1], vm[f])
        sm[f] = keep
    kf_start = np.arange(keyframes + 1) * frames_per_kf
    return palpix, thm, tvm, kf_start, pals, tile, pal, hm, vm, sm, W, H


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=8)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    palpix, thm, tvm, kf_start, pals, tile, pal, hm, vm, sm, W, H = workload(5, args.keyframes)
    F = int(kf_start[-1])
    threads = args.threads or min(16, len(os.sched_getaffinity(0)))
    # raw command bytes (what LZCompress receives), for the MB/s and the baseline
    raws = []
    for k in range(args.keyframes):
        f0, f1 = int(kf_start[k]), int(kf_start[k + 1])
        raws.append(gtm.keyframe_commands(tile[f0:f1], pal[f0:f1], hm[f0:f1], vm[f0:f1], sm[f0:f1], thm, tvm,
                                          pals[k]))
    raw = sum(map(len, raws)) + palpix.nbytes
    t0 = time.perf_counter()
    data = gtm.save_stream(palpix, thm, tvm, kf_start, pals, tile, pal, hm, vm, sm, W, H, 30.0, threads=threads)
    dt = time.perf_counter() - t0
    # single stream, single thread: the encoder's own rate
    t1 = time.perf_counter()
    one = gtm.lzma_encode(raws[1])
    dt1 = time.perf_counter() - t1
    # CPU comparator: liblzma (xz) on the same keyframe stream, FORMAT_ALONE (lc <= 4 there), preset 6
    t2 = time.perf_counter()
    xz = lzma.compress(raws[1], format=lzma.FORMAT_ALONE, filters=[{"id": lzma.FILTER_LZMA1, "preset": 6, "lc": 4,
                                                                      "lp": 0, "pb": 2, "dict_size": 1 << 21}])
    dt2 = time.perf_counter() - t2
    out = {"metric": "SaveStream MB/s (raw GTM command bytes -> .gtm)", "value": round(raw / dt / 1e6, 2),
           "unit": "MB/s", "threads": threads, "frames": F, "keyframes": args.keyframes,
           "raw_bytes": raw, "gtm_bytes": len(data), "ratio": round(len(data) / raw, 4),
           "frames_per_s": round(F / dt, 1),
           "single_stream": {"raw_bytes": len(raws[1]), "MB_s": round(len(raws[1]) / dt1 / 1e6, 2),
                             "bytes": len(one)},
           "cpu_comparator": {"kind": "liblzma preset 6, lc=4 (liblzma rejects lc=8 in .lzma), same stream",
                              "MB_s": round(len(raws[1]) / dt2 / 1e6, 2), "bytes": len(xz)},
           "config": {"workload": "C3 shape: 1920x1080 8x8, 24 frames per keyframe, 65536 reindexed tiles, "
                                  "128 palettes, 70 % of items smoothed (synthetic)"}}
    if args.check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import pyoracle
        from gtm_read import read_gtm
        g = read_gtm(pyoracle, data)
        ok = len(g.frames) == F and all(
            np.array_equal(items[:, 0] >= 0, ~sm[f].astype(bool)) for f, (items, _, _) in enumerate(g.frames))
        out["check"] = bool(ok)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

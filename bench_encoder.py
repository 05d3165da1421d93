#!/usr/bin/env python3
"""The encoder's whole FrameTiling pass over a clip, sustained (secondary line; the headline is bench.py).

btnDoFrameTilingClick (main.pas:945-977) over a C3-shaped clip: PrepareGlobalFT once, then for every keyframe
PrepareFrameTiling (UseOne's k = 8 preselection over the keyframe's distinct (PalIdx, GlobalTileIndex) items at
the requested quality, DoPsyV, the search index incl. ANN's kd-tree; main.pas:3791-3967), DoFrameTiling of its
frames (main.pas:3992-4047), then DoTemporalSmoothing of the keyframe (main.pas:4071-4119).  Every keyframe runs
every step (nothing is cached across keyframes); frames and tilemaps are resident in HBM (generated on the GPU
before timing).  With --overlap (default) keyframe k+1's Prepare runs on a second stream, in a second host thread,
while keyframe k's FrameTiling and Smooth run.

Synthetic clip (SURVEY.md 8(d) shapes): 1080p, 24-frame keyframes (1000 frames = 41 x 24 + 16), frame tiles with the
bench's mix (50 % gradients, 30 % texture, 20 % flat; 30 % of tiles re-drawn per frame), a 64k tileset with 20 %
mirror-symmetric tiles, 128 palettes and their centroids; each frame tile's tilemap item before FrameTiling is a
tileset tile (re-drawn with the frame tile) in that tile's palette (its DitheringPalIndex bin).  One keyframe is
re-checked against the CPU restatement after the timed region: UseOne's used table (oracle mark_used, ANN's k = 8
order), the candidate count, a sample of its FrameTiling items, and a column subset of its Smooth.

Prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F16_TFLOPS = 2500.0   # MI355X dense fp16 MFMA (MI355X_MICROARCH.md; sparsity excluded)
GENERIC_KERNEL = "nn_shortlist16_kernel<S=6,L=4,CB=8,NW=8,QB=4>"


def frame_tiles_gpu(torch, g, n, dev):
    """synth.frame_tiles' mix on the GPU: [n, 64] int32 0x00BBGGRR."""
    kind = torch.rand(n, generator=g, device=dev)
    yy, xx = torch.meshgrid(torch.arange(8, device=dev), torch.arange(8, device=dev), indexing="ij")
    xx = (xx.reshape(64) / 7.0).double()
    yy = (yy.reshape(64) / 7.0).double()
    c0 = torch.randint(0, 256, (n, 1, 3), generator=g, device=dev).double()
    c1 = torch.randint(0, 256, (n, 1, 3), generator=g, device=dev).double()
    ang = torch.rand((n, 1, 1), generator=g, device=dev, dtype=torch.float64) * 2 * np.pi
    t = torch.cos(ang) * xx[None, :, None] + torch.sin(ang) * yy[None, :, None]
    t = (t - t.amin(1, keepdim=True)) / (t.amax(1, keepdim=True) - t.amin(1, keepdim=True)).clamp_min(1e-9)
    grad = c0 + (c1 - c0) * t
    mean = torch.randint(32, 224, (n, 1, 3), generator=g, device=dev).double()
    tex = mean + torch.randint(-32, 33, (n, 64, 3), generator=g, device=dev).double()
    flat = torch.randint(0, 256, (n, 1, 3), generator=g, device=dev).double().expand(n, 64, 3)
    k = kind[:, None, None]
    out = torch.where(k < 0.5, grad, torch.where(k < 0.8, tex, flat))
    px = out.round().clamp(0, 255).int()
    return (px[..., 2] << 16) | (px[..., 1] << 8) | px[..., 0]


def keyframe_gpu(torch, g, F, Q, T, dev, change=0.3, subset=0):
    """[F, Q, 64] frames and [F, Q] tilemap items (tileset tiles; an item is re-drawn with its frame tile).
    subset > 0: the keyframe's items come from `subset` random tiles of the set (a shot uses part of the tileset)."""
    fr = torch.empty((F, Q, 64), dtype=torch.int32, device=dev)
    it = torch.empty((F, Q), dtype=torch.int32, device=dev)
    pool = torch.randperm(T, generator=g, device=dev)[:subset].int() if subset else None
    draw = (lambda n: pool[torch.randint(0, subset, (n,), generator=g, device=dev)]) if subset else \
        (lambda n: torch.randint(0, T, (n,), generator=g, device=dev, dtype=torch.int32))
    fr[0] = frame_tiles_gpu(torch, g, Q, dev)
    it[0] = draw(Q)
    for f in range(1, F):
        sel = torch.rand(Q, generator=g, device=dev) < change
        fr[f] = fr[f - 1]
        it[f] = it[f - 1]
        n = int(sel.sum().item())
        fr[f][sel] = frame_tiles_gpu(torch, g, n, dev)
        it[f][sel] = draw(n)
    return fr, it


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--kf-len", type=int, default=24)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tileset", type=int, default=65536)
    ap.add_argument("--palettes", type=int, default=128)
    ap.add_argument("--quality", type=int, default=1, help="0 Fast, 1 Medium (the reference default), 2 Slow")
    ap.add_argument("--item-tiles", type=int, default=0,
                    help="tiles a keyframe's items are drawn from (0: the whole tileset, uniformly)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--prep-priority", type=int, default=1,
                    help="1: the next keyframe's Prepare on a high-priority stream (its short kernels and host syncs "
                         "then get CUs as FrameTiling's workgroups retire instead of after the whole grid); 0: normal")
    ap.add_argument("--no-smooth", action="store_true")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1: keyframe k + 1's FrameTiling queued behind k's as soon as its Prepare ends, Smooth on a third "
                         "stream, handles closed by a closer thread (A/B study: whole tileset +1 %%, shot-local -4 %%, "
                         "profiles/r06/pp_encoder_pipeline_ab.txt); 0: the host waits for each keyframe before the next")
    ap.add_argument("--async-close", type=int, default=1,
                    help="1: the previous keyframe's handle is closed by a closer thread (its device-wide synchronisation "
                         "and block filing off the host path between two keyframes: +0.7 %% both item modes, "
                         "profiles/r06/ac_encoder_async_close_ab.txt); 0: closed before the next launch")
    ap.add_argument("--check-kf", type=int, default=1, help="keyframe re-checked against the restatement (-1: none)")
    ap.add_argument("--check-queries", type=int, default=1500)
    ap.add_argument("--check-items", type=int, default=1000, help="items whose k = 8 search is re-checked")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host cores this process may use (benchutil)")
    ap.add_argument("--seed", type=int, default=20261017)
    ap.add_argument("--lib", default="", help="a libANN.so build to load instead of tiler_amd/lib/libANN.so (A/B)")
    return ap


def run(args) -> dict:
    """The sustained clip; also bench.py's `secondary.encoder_*` lines."""
    import torch

    import tiler_amd
    from tiler_amd import frame_tiling as ftm
    from tiler_amd import synth
    from tiler_amd._lib import check

    if getattr(args, "lib", ""):
        import tiler_amd._lib as _l
        _l.LIB_PATH = os.path.abspath(args.lib)
    lib = tiler_amd.load()
    devi = torch.cuda.current_device() if torch.cuda.is_initialized() else 0
    check(lib.tiler_init(devi), "tiler_init")
    dev = torch.device("cuda", devi)
    vp = ctypes.c_void_p
    W, H, T, P = args.width, args.height, args.tileset, args.palettes
    Q = (W // 8) * (H // 8)
    starts = list(range(0, args.frames, args.kf_len)) + [args.frames]
    nkf = len(starts) - 1

    # ---- inputs (untimed): tileset, palettes, centroids; every keyframe's frames + items generated in HBM ----
    rng = np.random.default_rng(args.seed)
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    tile_pal = rng.integers(0, P, T).astype(np.int32)
    cents = synth.palette_centroids(pals)
    near = ftm.near_palettes(cents) if args.quality == ftm.FT_MEDIUM else None
    d_tiles = torch.from_numpy(tiles).to(dev)
    d_thm = torch.from_numpy(thm).to(dev)
    d_tvm = torch.from_numpy(tvm).to(dev)
    d_pals = torch.from_numpy(pals).to(dev)
    d_tpal = torch.from_numpy(tile_pal).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed)
    frames, items_t, items_p = [], [], []
    for k in range(nkf):
        fr, it = keyframe_gpu(torch, g, starts[k + 1] - starts[k], Q, T, dev, subset=args.item_tiles)
        frames.append(fr)
        items_t.append(it)
        items_p.append(d_tpal[it.long()].int())
    torch.cuda.synchronize(dev)
    print(f"[bench_encoder] {args.frames} frames x {Q} tiles in HBM, {nkf} keyframes", file=sys.stderr, flush=True)

    s_ft = torch.cuda.Stream(dev)     # FrameTiling + Smooth
    # PrepareFrameTiling of the next keyframe; high priority (torch: negative = higher) by default
    s_prep = torch.cuda.Stream(dev, priority=-1) if args.prep_priority else torch.cuda.Stream(dev)
    outs = []
    for k in range(nkf):
        n = (starts[k + 1] - starts[k]) * Q
        outs.append({nm: torch.empty(n, dtype=dt, device=dev) for nm, dt in
                     (("tile", torch.int32), ("pal", torch.int32), ("hm", torch.uint8), ("vm", torch.uint8),
                      ("err", torch.float32))})
    sm = [None] * nkf
    times = {"prepare": [], "ft_smooth": [], "close": [], "join": [], "prep_call": []}
    stats_kf = {}
    info_all = []

    def prepare(k, gds, stream):
        t0 = time.perf_counter()
        kt, info = ftm.prepare_frame_tiling_dev(gds, items_t[k].data_ptr(), items_p[k].data_ptr(), items_t[k].numel(),
                                                d_tiles.data_ptr(), d_thm.data_ptr(), d_tvm.data_ptr(), T,
                                                d_pals.data_ptr(), P, args.quality, near, True, -1,
                                                stream.cuda_stream)
        times["prep_call"].append(time.perf_counter() - t0)
        stream.synchronize()
        times["prepare"].append(time.perf_counter() - t0)
        info_all.append(info)
        return kt

    def ft_smooth(k, kt):
        t0 = time.perf_counter()
        o = outs[k]
        F = starts[k + 1] - starts[k]
        n = F * Q
        check(lib.tiler_frame_tiling_dev(kt.handle, vp(frames[k].data_ptr()), n, 1, -1, vp(o["tile"].data_ptr()),
                                         vp(o["pal"].data_ptr()), vp(o["hm"].data_ptr()), vp(o["vm"].data_ptr()),
                                         vp(o["err"].data_ptr()), vp(s_ft.cuda_stream)), "tiler_frame_tiling_dev")
        if not args.no_smooth:
            with torch.cuda.stream(s_ft):
                st = {nm: o[nm].view(F, Q).clone() for nm in ("tile", "pal", "hm", "vm")}
                st["smoothed"] = torch.zeros((F, Q), dtype=torch.uint8, device=dev)
            check(lib.tiler_smooth_keyframe_dev(F, Q, vp(st["tile"].data_ptr()), None, vp(st["pal"].data_ptr()),
                                                vp(st["hm"].data_ptr()), vp(st["vm"].data_ptr()),
                                                vp(st["smoothed"].data_ptr()), vp(d_tiles.data_ptr()),
                                                vp(d_pals.data_ptr()), 0.02, vp(s_ft.cuda_stream)),
                  "tiler_smooth_keyframe_dev")
            sm[k] = st
        s_ft.synchronize()
        times["ft_smooth"].append(time.perf_counter() - t0)
        if k == args.check_kf or (k == 0 and args.check_kf < 0):
            stats_kf.update(kt.stats())

    kept = {}
    s_sm = torch.cuda.Stream(dev)  # --pipeline: keyframe k's Smooth, beside keyframe k + 1's FrameTiling

    def run_pipelined(gds, keep):
        """FrameTiling k + 1 is queued on its stream behind FrameTiling k as soon as Prepare k + 1 has ended, so the GPU
        does not wait for the host between keyframes; Smooth k runs on a third stream once FrameTiling k's event has
        fired (its host sync then waits for k alone); a finished keyframe's handle is closed by a closer thread (the
        close synchronises the device before filing the handle's blocks, which would otherwise hold up the queueing)."""
        nonlocal_ft = {}
        box = {}
        closing = []
        closer_go = threading.Event()
        closer_stop = [False]

        def closer():
            while True:
                closer_go.wait()
                closer_go.clear()
                while closing:
                    closing.pop(0).close()
                if closer_stop[0] and not closing:
                    return

        ct = threading.Thread(target=closer)
        ct.start()

        def launch_ft(k, kt):
            o = outs[k]
            n = (starts[k + 1] - starts[k]) * Q
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s_ft)
            check(lib.tiler_frame_tiling_dev(kt.handle, vp(frames[k].data_ptr()), n, 1, -1, vp(o["tile"].data_ptr()),
                                             vp(o["pal"].data_ptr()), vp(o["hm"].data_ptr()), vp(o["vm"].data_ptr()),
                                             vp(o["err"].data_ptr()), vp(s_ft.cuda_stream)), "tiler_frame_tiling_dev")
            e1.record(s_ft)
            nonlocal_ft[k] = (e0, e1)

        def smooth(k):
            F = starts[k + 1] - starts[k]
            o = outs[k]
            e0, e1 = nonlocal_ft[k]
            s_sm.wait_event(e1)
            es0 = torch.cuda.Event(enable_timing=True)
            es1 = torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s_sm):
                es0.record(s_sm)
                st = {nm: o[nm].view(F, Q).clone() for nm in ("tile", "pal", "hm", "vm")}
                st["smoothed"] = torch.zeros((F, Q), dtype=torch.uint8, device=dev)
            check(lib.tiler_smooth_keyframe_dev(F, Q, vp(st["tile"].data_ptr()), None, vp(st["pal"].data_ptr()),
                                                vp(st["hm"].data_ptr()), vp(st["vm"].data_ptr()),
                                                vp(st["smoothed"].data_ptr()), vp(d_tiles.data_ptr()),
                                                vp(d_pals.data_ptr()), 0.02, vp(s_sm.cuda_stream)),
                  "tiler_smooth_keyframe_dev")
            es1.record(s_sm)
            sm[k] = st
            return es0, es1

        def start_prep(k1):
            if k1 < nkf:
                w = threading.Thread(target=lambda: box.__setitem__(k1, prepare(k1, gds, s_prep)))
                w.start()
                return w
            return None

        w = start_prep(0)
        w.join()
        kts = {0: box.pop(0)}
        w = start_prep(1)
        launch_ft(0, kts[0])
        for k in range(nkf):
            if k + 1 < nkf:
                tj = time.perf_counter()
                w.join()
                times["join"].append(time.perf_counter() - tj)
                kts[k + 1] = box.pop(k + 1)
                w = start_prep(k + 2)  # before the launch: FrameTiling k + 1 may wait on the host for k's end
                launch_ft(k + 1, kts[k + 1])
            if not args.no_smooth:
                es = smooth(k)
            e0, e1 = nonlocal_ft[k]
            e1.synchronize()
            t_ft = e0.elapsed_time(e1)
            if not args.no_smooth:
                es[1].synchronize()
                t_ft += es[0].elapsed_time(es[1])
            times["ft_smooth"].append(t_ft * 1e-3)
            kt = kts.pop(k)
            if k == args.check_kf or (k == 0 and args.check_kf < 0):
                stats_kf.update(kt.stats())
            if k == args.check_kf and keep:
                kept["kt"] = kt
            else:
                closing.append(kt)
                closer_go.set()
        closer_stop[0] = True
        closer_go.set()
        ct.join()

    def run_clip(keep=False):
        for v in times.values():
            v.clear()
        info_all.clear()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        gds = ftm.prepare_global_ft(tiles)  # PrepareGlobalFT, once per pass (main.pas:3736-3780)
        t_global = time.perf_counter() - t0
        if args.no_overlap:
            for k in range(nkf):
                kt = prepare(k, gds, s_prep)
                ft_smooth(k, kt)
                if k == args.check_kf and keep:
                    kept["kt"] = kt
                else:
                    kt.close()
        elif args.pipeline:
            run_pipelined(gds, keep)
        else:
            box = {}
            worker = threading.Thread(target=lambda: box.__setitem__(0, prepare(0, gds, s_prep)))
            worker.start()
            prev = None
            closers = []
            for k in range(nkf):
                tj = time.perf_counter()
                worker.join()
                times["join"].append(time.perf_counter() - tj)
                kt = box.pop(k)
                tc = time.perf_counter()
                if prev is not None and prev is not kept.get("kt"):
                    if args.async_close:  # the close waits for the device, so not on the launching thread
                        closers.append(threading.Thread(target=prev.close))
                        closers[-1].start()
                    else:
                        prev.close()  # keyframe k-1 is finished and nothing else is in flight: its frees cost nothing
                times["close"].append(time.perf_counter() - tc)
                if k + 1 < nkf:
                    worker = threading.Thread(target=lambda k1=k + 1: box.__setitem__(k1, prepare(k1, gds, s_prep)))
                    worker.start()
                ft_smooth(k, kt)
                if k == args.check_kf and keep:
                    kept["kt"] = kt  # the re-checked keyframe's candidate set is read back after the timed region
                prev = kt
            for c in closers:
                c.join()
            if prev is not kept.get("kt"):
                prev.close()
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        gds.kdt.close()
        return wall, t_global

    def kernel_times():
        names = ("psyv", "nn_prep", "nn_shortlist", "nn_orbit", "nn_rescore", "nn_pairs", "nn_collect", "nn_rescore2",
                 "nn_exact", "kd_verify", "kd_replay", "smooth")
        out = {}
        for nm in names:
            n = ctypes.c_int(0)
            ms = lib.tiler_timing_get(nm.encode(), ctypes.byref(n))
            if n.value:
                out[nm] = {"ms": round(ms, 3), "launches": n.value}
        return out

    # diagnostics (untimed): one keyframe's Prepare with per-kernel times and the k = 8 search's tier counts, then its
    # FrameTiling + Smooth the same way
    gds0 = ftm.prepare_global_ft(tiles)
    prepare(0, gds0, s_prep)  # warm
    info_all.clear()
    times["prepare"].clear()
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    kt0 = prepare(0, gds0, s_prep)
    lib.tiler_timing_enable(0)
    diag = {"prepare_ms": round(1e3 * times["prepare"][-1], 3), "prepare_kernels": kernel_times(),
            "knn8_search_stats": gds0.kdt.stats(), "items": info_all[-1]["items"],
            "candidates": info_all[-1]["candidates"], "kd_build_ms": kt0.stats().get("kd_build_ms")}
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    ft_smooth(0, kt0)
    lib.tiler_timing_enable(0)
    diag["ft_smooth_ms"] = round(1e3 * times["ft_smooth"][-1], 3)
    diag["ft_kernels"] = kernel_times()
    diag["ft_search_stats"] = kt0.stats()
    kt0.close()
    gds0.kdt.close()
    times["prepare"].clear()
    times["ft_smooth"].clear()
    info_all.clear()
    print("[bench_encoder] diag " + json.dumps(diag), file=sys.stderr, flush=True)

    # one untimed pass on the first keyframes (allocations, code objects), then the timed clip
    warm_n = min(2, nkf)
    _nkf = nkf
    nkf = warm_n
    run_clip()
    nkf = _nkf
    print("[bench_encoder] warm-up pass done", file=sys.stderr, flush=True)
    wall, t_global = run_clip(keep=True)
    print(f"[bench_encoder] clip: {wall:.3f} s", file=sys.stderr, flush=True)
    tiles_total = args.frames * Q
    value = tiles_total / wall / 1e6
    cand = [i["candidates"] for i in info_all]
    res = {"metric": "sustained FrameTiling Mtiles/s over a clip incl. PrepareGlobalFT + per-keyframe "
                     "PrepareFrameTiling + Smooth", "value": round(value, 3), "unit": "Mtiles/s",
           "wall_s": round(wall, 4), "frames": args.frames, "keyframes": nkf, "tiles": tiles_total,
           "overlap": not args.no_overlap, "prep_priority": args.prep_priority, "quality": ["fast", "medium", "slow"][args.quality],
           "prepare_global_ms": round(t_global * 1e3, 2),
           "prepare_ms_avg": round(1e3 * float(np.mean(times["prepare"])), 3),
           "ft_smooth_ms_avg": round(1e3 * float(np.mean(times["ft_smooth"])), 3),
           "loop_ms_avg": {k: round(1e3 * float(np.mean(times[k])), 3) for k in ("join", "close", "prep_call") if times[k]},
           "items_avg": round(float(np.mean([i["items"] for i in info_all])), 1),
           "candidates_avg": round(float(np.mean(cand)), 1), "candidates_min": int(min(cand)),
           "candidates_max": int(max(cand)), "search_stats_one_keyframe": stats_kf,
           "data": "synthetic, generated in HBM before timing",
           "config": {"workload": f"{W}x{H}, {args.frames} frames, {args.kf_len}-frame keyframes, {T}-tile set, "
                                  f"{P} palettes, items from "
                                  f"{args.item_tiles or T} tiles per keyframe"}}

    res["diag"] = diag
    # roofline of the FrameTiling search kernel on keyframe 0 (diag, HIP events on its stream): the generic 16x16x32
    # shortlist issues 2*M*D flops per query (M = the keyframe's candidates, D = 192; real candidate sets have no
    # mirror-orbit structure); flat query tiles grouped last issue only k-step 0 (flat_queries)
    fk = diag["ft_kernels"]
    orbit_kf = bool(diag.get("ft_search_stats", {}).get("orbit_search"))
    sl = fk.get("nn_orbit" if orbit_kf else "nn_shortlist")
    q0 = (starts[1] - starts[0]) * Q
    m0 = diag["candidates"]
    if sl and not orbit_kf:
        nflat = diag.get("ft_search_stats", {}).get("flat_queries", 0) or 0
        s16 = 6
        flops = 2.0 * (-(-m0 // 16) * 16) * 32 * (s16 * (q0 - nflat) + nflat)
        ach = flops / (sl["ms"] * 1e-3) / 1e12
        res["roofline"] = {"bound": "mfma", "kernel": GENERIC_KERNEL, "achieved": round(ach, 2), "peak": PEAK_F16_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(ach / PEAK_F16_TFLOPS, 4), "kernel_ms": sl["ms"],
                           "flops_per_launch": flops, "queries": q0, "flat_queries": nflat, "candidates": m0,
                           "bruteforce_flops": 2.0 * m0 * 192 * q0,
                           "note": "issued MFMA flops (candidates padded to 16-row blocks; 6 k-steps of 32 per query, "
                                   "1 for flat query tiles grouped last) / the kernel's HIP-event time on keyframe 0; "
                                   "dense fp16 peak"}
    elif sl:
        res["roofline"] = {"bound": "mfma", "kernel": "nn_orbit_shortlist_pipe_kernel", "kernel_ms": sl["ms"],
                           "note": "orbit path (candidate set with mirror orbits)"}
    import hashlib
    hsh = hashlib.blake2b(digest_size=8)
    for k in range(nkf):  # every keyframe's FrameTiling items + errors (equal digest = identical outputs)
        for nm in ("tile", "pal", "hm", "vm", "err"):
            hsh.update(outs[k][nm].cpu().numpy().tobytes())
    res["out_digest"] = hsh.hexdigest()
    print("[bench_encoder] " + json.dumps({k: res[k] for k in ("value", "wall_s", "prepare_ms_avg", "ft_smooth_ms_avg",
                                                                "items_avg", "candidates_avg", "out_digest")}), file=sys.stderr,
          flush=True)

    # ---- re-check one keyframe against the CPU restatement (after the timed region), bounded ----
    # The reference's Prepare (UseOne's k = 8 kd search of every item in 64-d, main.pas:3830) takes minutes on the
    # host, so the chain is checked link by link: (1) the k = 8 search of a sample of the keyframe's items against the
    # restated ANN search; (2) the device Prepare's candidate set (tiler_ft_get_maps on the keyframe's own handle from
    # the timed run) against the host UseOne over the k = 8 results of ALL the keyframe's items (frame_tiling.mark_used,
    # DoPsyV emission order) -- every used cell, in order; (3) a sample of its FrameTiling items against the restated
    # ANN search over THAT candidate set (the CPU rate is timed here); (4) a column sample of its Smooth.
    ck = args.check_kf
    if 0 <= ck < nkf and "kt" in kept:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as oracle
        from benchutil import host_cores
        threads = args.cpu_threads or host_cores()["usable"]
        t0 = time.perf_counter()
        say = lambda m: print(f"[bench_encoder] check: {m} ({time.perf_counter() - t0:.1f} s)", file=sys.stderr,
                              flush=True)  # noqa: E731
        kt_ck = kept.pop("kt")
        g_tile, g_pal, g_attr = kt_ck.maps()
        kt_ck.close()
        it = items_t[ck].cpu().numpy().ravel()
        ip = items_p[ck].cpu().numpy().ravel()
        chk = {"keyframe": ck, "candidates_gpu": int(g_tile.size)}
        # (1) k = 8 searches of sampled distinct items, GPU (batched, same global handle kind) vs restated ANN
        gdsc = ftm.prepare_global_ft(tiles)
        keys = np.unique(ip.astype(np.int64) * T + it.astype(np.int64))
        ks = np.random.default_rng(4).choice(keys, min(args.check_items, keys.size), replace=False)
        qk = tiles[(ks % T)].astype(np.float32)
        gi8, ge8 = gdsc.kdt.search_batch(qk, k=8)
        o_ds, _, _ = oracle.prepare_global_ds(tiles)
        okd = oracle.KDTree(o_ds)
        oi8, oe8 = okd.search_batch(qk, threads=threads, k=8)
        okd.close()
        chk["knn8_items"] = int(ks.size)
        chk["knn8_mismatches"] = int(np.count_nonzero(np.any((gi8 != oi8) | (ge8.view(np.uint32) !=
                                                                          oe8.view(np.uint32)), axis=1)))
        say("k = 8 sample")
        # (2) the whole candidate set: host UseOne over the k = 8 results of every item vs the device Prepare
        corrs, highest = ftm.palette_corr(cents)
        used = ftm.mark_used(gdsc, tiles, ip, it, P, args.quality, corrs, highest)
        gdsc.kdt.close()
        hds = synth.ft_dataset_from_used(used, thm, tvm)
        chk["candidates_host"] = int(hds.tile_of.size)
        chk["candidate_set_equal"] = bool(np.array_equal(hds.tile_of, g_tile) and np.array_equal(hds.pal_of, g_pal)
                                          and np.array_equal(hds.attrs, g_attr))
        say("candidate set")
        # (3) FrameTiling items vs the restated search over the device's candidate set
        used_g = np.zeros((P, T, 4), np.uint8)
        used_g[g_pal, g_tile, g_attr] = 1
        ods, ot, op, oa = oracle.build_ft_dataset(used_g, tiles, thm, tvm, pals)
        fr = frames[ck].cpu().numpy().reshape(-1, 64)
        pick = np.random.default_rng(5).choice(fr.shape[0], min(args.check_queries, fr.shape[0]), replace=False)
        t1 = time.perf_counter()
        okd = oracle.KDTree(ods)
        build_s = time.perf_counter() - t1
        t1 = time.perf_counter()
        qd = oracle.psyv_batch(pick.size, rgb=fr[pick], flags=2).astype(np.float32)
        ki, ke = okd.search_batch(qd, threads=threads)
        cpu_s = time.perf_counter() - t1
        okd.close()
        go = {nm: outs[ck][nm].cpu().numpy() for nm in ("tile", "pal", "hm", "vm", "err")}
        mism = int(np.count_nonzero((go["tile"][pick] != ot[ki]) | (go["pal"][pick] != op[ki]) |
                                    (go["hm"][pick] != (oa[ki] & 1)) | (go["vm"][pick] != (oa[ki] >> 1)) |
                                    (go["err"][pick].view(np.uint32) != ke.view(np.uint32))))
        chk["ft_queries"] = int(pick.size)
        chk["ft_mismatches"] = mism
        res["cpu_baseline"] = {"value": round(pick.size / cpu_s / 1e6, 6), "unit": "Mtiles/s", "cores": threads,
                               "kind": "port",
                               "sample": f"{pick.size} frame tiles of keyframe {ck} vs its {ods.shape[0]} candidates: "
                                         f"fp64 descriptor + ANN 1.1.2 kd-tree search (oracle/ann_kdtree.c, ANN_KD_STD, "
                                         f"bucket 1, eps 0), tree build {build_s:.1f} s untimed, {threads} threads; "
                                         f"the per-keyframe Prepare and Smooth are not in this rate"}
        say("frame tiling")
        if sm[ck] is not None:
            F = starts[ck + 1] - starts[ck]
            cols = np.sort(np.random.default_rng(6).choice(Q, min(2000, Q), replace=False))
            sub = lambda a: np.ascontiguousarray(a.reshape(F, Q)[:, cols])  # noqa: E731
            so = oracle.smooth(sub(go["tile"]), sub(go["pal"]), sub(go["hm"]), sub(go["vm"]),
                               np.zeros((F, cols.size), np.uint8), tiles, pals, 0.02)
            gs = [sub(sm[ck][nm].cpu().numpy()) for nm in ("tile", "pal", "hm", "vm", "smoothed")]
            chk["smooth_positions"] = int(cols.size)
            chk["smooth_mismatches"] = int(sum(np.count_nonzero(a != b) for a, b in zip(gs, so)))
        chk["check_s"] = round(time.perf_counter() - t0, 2)
        chk["mismatches_total"] = (chk["knn8_mismatches"] + chk["ft_mismatches"] + chk.get("smooth_mismatches", 0) +
                                   (0 if chk["candidate_set_equal"] else 1))
        res["parity"] = chk
    for k in range(nkf):
        sm[k] = None
    outs.clear()
    frames.clear()
    items_t.clear()
    items_p.clear()
    return res


if __name__ == "__main__":
    print(json.dumps(run(parser().parse_args())), flush=True)

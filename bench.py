#!/usr/bin/env python3
"""FrameTiling throughput on MI355X (BASELINE.json metric), one process per GPU.

A step = DoFrameTiling (main.pas:3992-4047) over one keyframe batch of synthetic 1080p frames:
query PsyV descriptors (fp64 Haar -> fp32) + exact NN against the keyframe's 262,144 mirror
candidates of a 64k tileset + tilemap items, all inputs resident in HBM before timing starts.
Weak scaling: every rank tiles its own keyframe (keyframes are independent, main.pas:4005-4011);
there is no data-path collective.  The tileset is broadcast once from rank 0 (RCCL) before timing.

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the
dominant kernel (nn_shortlist: MFMA) and a bounded `cpu_baseline` of the oracle on the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FrameTiling Mtiles/sec @1080p 8×8, 64k tileset; % HBM roofline at 1/2/4/8 GPU"
PEAK_F16_TFLOPS = 2500.0   # MI355X dense fp16 MFMA (MI355X_MICROARCH.md; sparsity excluded)
ORBIT_KERNEL = "nn_orbit_shortlist_pipe_kernel<L=4,CB=4,NW=8,QB=2>"
GENERIC_KERNEL = "nn_shortlist16_kernel<S=6,L=4,CB=8,NW=8,QB=4>"
PEAK_HBM_GBS = 8000.0
FT_BYTES_PER_TILE_FIXED = 256 + 8 + 4   # RGB in + tilemap item + err out (+ candidate stream / Q_KF)

CONFIGS = {
    # name: (width, height, frames per keyframe step, tileset size)
    "c3": (1920, 1080, 24, 65536),
    "c2": (1280, 720, 24, 16384),
    "c5": (3840, 2160, 24, 262144),
    "tiny": (320, 240, 4, 2048),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline budget (rank 0)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host cores this process may use "
                    "(benchutil.host_cores: affinity mask, cgroup quota, the box's advertised share)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-smooth", action="store_true")
    ap.add_argument("--no-keyframes", action="store_true")
    ap.add_argument("--no-dither", action="store_true")
    ap.add_argument("--no-globaltiling", action="store_true", help="skip the C4 K-Modes secondary line")
    ap.add_argument("--no-palettes", action="store_true", help="skip the palette-generation secondary line")
    ap.add_argument("--no-encoder", action="store_true", help="skip the sustained 1000-frame encoder lines")
    ap.add_argument("--no-per-call", action="store_true", help="skip the per-tile ann_kdtree_search line")
    ap.add_argument("--per-call-queries", type=int, default=8192)
    ap.add_argument("--palette-frames", type=int, default=8, help="frames per keyframe of the palette lines")
    ap.add_argument("--palette-keyframes", type=int, default=8,
                    help="keyframes of the clip-level palette line (all pairs in one call; <= 1: skip it)")
    ap.add_argument("--clip-frames", type=int, default=1000, help="keyframe-detection clip length (C3: 1000)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL over xGMI, the product); gloo only to rehearse the N>1 control flow")
    ap.add_argument("--rank-check", action="store_true",
                    help="launcher self-test without a GPU: the ranks rendezvous over gloo, all-reduce their ranks "
                         "and rank 0 prints the world it saw (tests/test_bench_launch.py)")
    args = ap.parse_args()

    # --gpus N: one process per GPU.  Under an external launcher (torch.distributed.run) WORLD_SIZE must agree;
    # without one this process starts the N ranks itself BEFORE touching the GPU and relays rank 0's line.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}: refusing to time a different world",
              file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    if args.rank_check:
        return rank_check()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # TILER_BENCH_ONE_DEVICE=1: every rank on cuda:0 (rehearsal of the N>1 path on a one-GPU box, gloo)
    devi = 0 if os.environ.get("TILER_BENCH_ONE_DEVICE") == "1" else local
    # under a launcher the process group is made even at WORLD_SIZE=1, so the RCCL branch (broadcast, barriers, the
    # max-over-ranks all-reduce) is the one that runs; a bare `python bench.py` stays single-process
    use_dist = env_world is not None
    if use_dist:
        torch.cuda.set_device(devi)
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", devi)
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # where collectives' tensors live

    import tiler_amd
    from tiler_amd import synth
    from tiler_amd._lib import check

    lib = tiler_amd.load()
    check(lib.tiler_init(devi), "tiler_init")

    W, H, F, TS = CONFIGS[args.config]
    Q = (W // 8) * (H // 8)
    P = 128

    # ---- global tileset + palettes: generated on rank 0, all-gathered (broadcast) over RCCL ----
    rng0 = np.random.default_rng(args.seed)
    if rank == 0:
        pals = synth.palettes(rng0, P)
        tiles, thm, tvm = synth.tileset(rng0, TS)
        tile_pal = rng0.integers(0, P, TS).astype(np.int32)
        packed = np.concatenate([tiles.reshape(-1).astype(np.int32), thm.astype(np.int32), tvm.astype(np.int32),
                                 tile_pal, pals.reshape(-1)])
        t_packed = torch.from_numpy(packed).to(cdev)
    else:
        t_packed = torch.empty(TS * 64 + 3 * TS + P * 16, dtype=torch.int32, device=cdev)
    if use_dist:
        dist.broadcast(t_packed, 0)
    packed = t_packed.cpu().numpy()
    o = 0
    tiles = packed[o:o + TS * 64].astype(np.uint8).reshape(TS, 64); o += TS * 64
    thm = packed[o:o + TS].astype(np.uint8); o += TS
    tvm = packed[o:o + TS].astype(np.uint8); o += TS
    tile_pal = packed[o:o + TS].astype(np.int32); o += TS
    pals = packed[o:o + P * 16].astype(np.int32).reshape(P, 16)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(tile_pal, P), thm, tvm)
    M = ds.tile_of.size

    # ---- this rank's keyframe (independent seed per rank) ----
    rng = np.random.default_rng(args.seed + 1 + rank)
    frames = synth.keyframe_frames(rng, F, Q)
    d_rgb = torch.from_numpy(frames.reshape(-1, 64)).to(dev)
    QK = d_rgb.shape[0]

    # ---- keyframe dataset in HBM: candidate descriptors on the GPU (DoPsyV) + index ----
    stream = torch.cuda.current_stream(dev).cuda_stream
    d_tiles = torch.from_numpy(tiles).to(dev)
    d_pals = torch.from_numpy(pals).to(dev)
    d_to = torch.from_numpy(ds.tile_of).to(dev)
    d_po = torch.from_numpy(ds.pal_of).to(dev)
    d_fl = torch.from_numpy(ds.psyv_flags).to(dev)
    import ctypes
    vp = ctypes.c_void_p

    def prepare():
        """PrepareFrameTiling's DoPsyV + DoBuild for the keyframe (main.pas:3883-3967): candidate descriptors
        on the GPU, then the search index (orbit grouping, fp16 fragments, norms) and the tilemap maps."""
        d_rows = torch.empty((M, 192), dtype=torch.float32, device=dev)
        tiler_amd.psyv_batch_dev(M, palpix=d_tiles.data_ptr(), tile_of=d_to.data_ptr(), palettes=d_pals.data_ptr(),
                                 pal_of=d_po.data_ptr(), flags_per=d_fl.data_ptr(), flags=1 | 2, gamma=-1,
                                 out32=d_rows.data_ptr(), stream=stream)
        torch.cuda.synchronize(dev)
        t = tiler_amd.KDTree(dev_ptr=d_rows.data_ptr(), n=M, dd=192, stream=stream)
        check(lib.tiler_ft_set_maps(t.handle, ds.tile_of.ctypes.data_as(vp), ds.pal_of.ctypes.data_as(vp),
                                    ds.attrs.ctypes.data_as(vp)), "tiler_ft_set_maps")
        torch.cuda.synchronize(dev)
        return t

    kdt = prepare()
    print(f"[bench] prepared {M} candidates", file=sys.stderr, flush=True)

    out_tile = torch.empty(QK, dtype=torch.int32, device=dev)
    out_pal = torch.empty(QK, dtype=torch.int32, device=dev)
    out_hm = torch.empty(QK, dtype=torch.uint8, device=dev)
    out_vm = torch.empty(QK, dtype=torch.uint8, device=dev)
    out_err = torch.empty(QK, dtype=torch.float32, device=dev)

    def step():
        check(lib.tiler_frame_tiling_dev(kdt.handle, vp(d_rgb.data_ptr()), QK, 1, -1, vp(out_tile.data_ptr()),
                                         vp(out_pal.data_ptr()), vp(out_hm.data_ptr()), vp(out_vm.data_ptr()),
                                         vp(out_err.data_ptr()), vp(stream)), "tiler_frame_tiling_dev")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    lib.tiler_timing_reset()
    lib.tiler_timing_enable(1)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    print(f"[bench] {args.steps} steps in {elapsed:.3f} s", file=sys.stderr, flush=True)
    lib.tiler_timing_enable(0)
    # digest of the last step's tilemap items and errors: A/B runs of kernel variants compare it (identical outputs)
    import hashlib
    hh = hashlib.sha256()
    for t_ in (out_tile, out_pal, out_hm, out_vm, out_err):
        hh.update(t_.cpu().numpy().tobytes())
    out_digest = hh.hexdigest()[:16]
    kernels = {}
    for name in ("psyv", "nn_prep", "nn_orbit", "nn_shortlist", "nn_rescore", "nn_pairs", "nn_collect", "nn_rescore2",
                 "nn_exact", "kd_verify", "kd_replay"):
        n = ctypes.c_int(0)
        ms = lib.tiler_timing_get(name.encode(), ctypes.byref(n))
        kernels[name] = {"ms_total": round(ms, 4), "launches": n.value,
                         "ms_avg": round(ms / n.value, 4) if n.value else None}
    stats = kdt.stats()
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ranks_seen = dist.get_world_size() if use_dist else 1
    total_tiles = QK * args.steps * ranks_seen
    value = total_tiles / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    # ---- roofline of the dominant kernel, per launch ----
    orbit = kernels["nn_orbit"]["launches"] > 0
    sl = kernels["nn_orbit"] if orbit else kernels["nn_shortlist"]
    sec = sl["ms_avg"] * 1e-3 if sl["ms_avg"] else None
    # launches of the dominant kernel per step: 2 when the search runs its query halves as two launches (orbit.hip
    # ORB_SPLIT_TAILS); the flops below are per launch, like the HIP-event and rocprofv3 per-dispatch times
    lps = max(1, round(sl["launches"] / args.steps)) if sl["launches"] else 1
    # the contraction this algorithm performs: the orbit kernel scores a tile's 4 mirrors with ONE 192-deep
    # fp16 contraction (2*G*D flops per query, G = tile orbits); the brute-force form is 2*M*D (M = candidates)
    # the MFMA work actually issued: k-steps of 16 dims x 32 groups per query (12 per block of groups; the blocks of
    # mirror-symmetric tiles skip their exactly-zero isotypic blocks: orbit_build / stats["orbit_ksteps"])
    ksteps = stats.get("orbit_ksteps") or 0
    nflat = stats.get("flat_queries") or 0  # flat tiles, grouped last: 3 k-steps per candidate block
    gblk = ((stats["orbit_groups"] or 0) + 31) // 32
    issued_launch = ((2.0 * 32 * 16 * (ksteps * (QK - nflat) + 3 * gblk * nflat)) if (orbit and ksteps) else
                     2.0 * (stats["orbit_groups"] if orbit else M) * 192 * QK) / lps
    bruteforce_launch = 2.0 * M * 192 * QK / lps
    issued = issued_launch / sec / 1e12 if sec else None
    effective = bruteforce_launch / sec / 1e12 if sec else None
    kname = "nn_orbit_shortlist_pipe_kernel" if orbit else "nn_shortlist16_kernel"
    traffic, traffic_src = pmc_traffic(kname)
    # the metric's own roofline: FrameTiling HBM bytes per matched tile (256 B RGB in + 12 B out +
    # the keyframe's candidate rows amortised over its queries, M*D*4 / Q_KF) over the step time
    ft_bytes_tile = FT_BYTES_PER_TILE_FIXED + M * 192 * 4 / QK
    hbm_gbs = ft_bytes_tile * QK * world / (ms_step * 1e-3) / 1e9
    roofline = {"bound": "mfma", "achieved": round(issued, 2) if issued else None, "peak": PEAK_F16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(issued / PEAK_F16_TFLOPS, 4) if issued else None,
                "traffic": traffic, "traffic_unit": "bytes/launch (HBM, FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": traffic_src, "kernel": ORBIT_KERNEL if orbit else GENERIC_KERNEL,
                "kernel_ms_avg": sl["ms_avg"], "launches_per_step": lps,
                "flops_per_launch": issued_launch,
                "effective_tflops": round(effective, 2) if effective else None,
                "effective_speedup": round(bruteforce_launch / issued_launch, 4),
                "hbm": {"bytes_per_tile": round(ft_bytes_tile, 1), "achieved_gbs": round(hbm_gbs, 2),
                        "peak_gbs": PEAK_HBM_GBS, "hbm_frac": round(hbm_gbs / PEAK_HBM_GBS, 6)},
                "issued_ksteps_per_query": ksteps, "flat_queries": nflat,
                "issued_ksteps_per_flat_query": 3 * gblk,
                "note": ("achieved/frac = MFMA flops the kernel issues (2*16*32 per k-step x the k-steps per query: "
                         "12 per block of 32 mirror orbits, fewer on the blocks of mirror-symmetric tiles whose zero "
                         "isotypic blocks are skipped, 3 per block for the flat query tiles grouped last; = 2*G*D "
                         "without them) / its "
                         "average launch time (HIP events on the launch stream) vs the dense fp16 peak -- per launch: "
                         "a step's search runs two query halves as two launches, the first half's rescore and pair "
                         "pass on a second stream beside the second launch, whose time includes that; "
                         "effective_tflops = the brute-force 2*M*D per query over the same time (effective_speedup = "
                         "brute-force / issued flops: the exact 4-mirror orbit algebra and the skipped zero blocks). hbm = the metric's '% HBM roofline': SURVEY.md 8(d) "
                         "bytes per matched tile x tiles / ms_per_step -- small by construction, the search is "
                         "MFMA-bound (SURVEY.md 7, hard part 5)")}
    # HBM-bound helpers: algorithmic bytes per launch / launch time.  "psyv" times the fused FrameTiling query
    # kernel (orbit_ft_query_kernel): 256 B RGB in; 768 B fp32 row + 384 B fp16 q' fragments + 32 B error
    # statistics + 4 B root-box distance out per tile
    for kn, bpt in (("psyv", 256 + 768 + 384 + 32 + 4),):
        kk = kernels.get(kn)
        if kk and kk["ms_avg"]:
            g = bpt * QK / (kk["ms_avg"] * 1e-3) / 1e9
            kk["hbm_gbs"] = round(g, 1)
            kk["hbm_frac"] = round(g / PEAK_HBM_GBS, 4)
            kk["bytes_per_launch"] = bpt * QK

    # ---- secondary: the keyframe's Prepare (reported separately from the FT step) ----
    prep = None
    if rank == 0:
        tps, kds = [], []
        for _ in range(3):  # steady state of an encoder walking keyframe after keyframe
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            kdt2 = prepare()
            tps.append(time.perf_counter() - t0)
            kds.append(kdt2.stats()["kd_build_ms"])
            kdt2.close()
        tp = min(tps)
        prep = {"ms": round(tp * 1e3, 3), "ms_each": [round(x * 1e3, 3) for x in tps], "candidates": M,
                "kd_build_ms_each": kds, "kd_levels": stats["kd_levels"],
                "what": "DoPsyV candidate descriptors (fp64 -> fp32 rows) + index build (ANN_KD_STD kd-tree for the "
                        "reference's tie order, mirror-orbit grouping, fp16 MFMA fragments, norms, maps), once per "
                        "keyframe, outside the FT step"}

    # ---- secondary (not the metric): Smooth over this keyframe's FT tilemap (DoTemporalSmoothing) ----
    smooth = None
    if rank == 0 and not args.no_smooth:
        tss = []
        lib.tiler_timing_reset()
        for rep_ in range(3):  # the first call also sets up the stream-ordered pool: report the best of 3
            s_tile = out_tile.view(F, Q).clone()
            s_pal = out_pal.view(F, Q).clone()
            s_hm, s_vm = out_hm.view(F, Q).clone(), out_vm.view(F, Q).clone()
            s_sm = torch.zeros((F, Q), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            lib.tiler_timing_enable(1 if rep_ > 0 else 0)
            t0 = time.perf_counter()
            check(lib.tiler_smooth_keyframe_dev(F, Q, vp(s_tile.data_ptr()), None, vp(s_pal.data_ptr()),
                                                vp(s_hm.data_ptr()), vp(s_vm.data_ptr()), vp(s_sm.data_ptr()),
                                                vp(d_tiles.data_ptr()), vp(d_pals.data_ptr()), 0.02, vp(stream)),
                  "tiler_smooth_keyframe_dev")
            torch.cuda.synchronize(dev)
            tss.append(time.perf_counter() - t0)
        lib.tiler_timing_enable(0)
        sm_parts = {}
        for kn in ("smooth_hash", "smooth_desc", "smooth_chain"):
            n_ = ctypes.c_int(0)
            ms_ = lib.tiler_timing_get(kn.encode(), ctypes.byref(n_))
            sm_parts[kn] = round(ms_ / n_.value, 4) if n_.value else None
        ts = min(tss)
        steps_s = (F - 1) * Q
        smooth = {"value": round(steps_s / ts / 1e6, 4), "unit": "Msteps/s", "ms": round(ts * 1e3, 3),
                  "ms_each": [round(x * 1e3, 3) for x in tss], "kernel_ms_avg": sm_parts,
                  "smoothed": int(s_sm.sum().item()), "shape": f"{F} frames x {Q} positions, Strength 0.02",
                  "hbm": {"bytes_per_step": 2 * 16 + 64 + 64,
                          "achieved_gbs": round(steps_s * (2 * 16 + 64 + 64) / ts / 1e9, 2),
                          "hbm_frac": round(steps_s * (2 * 16 + 64 + 64) / ts / 1e9 / PEAK_HBM_GBS, 6),
                          "note": "SURVEY.md 8(d) Smooth unit: 2 items + tile + palette per (position, frame) step "
                                  "(cache-resident; the chain is latency-bound)"}}
        if world == 1 and not args.no_cpu:
            # DoTemporalSmoothing on the host (oracle/tiler_oracle.c or_smooth: scalar fp64, positions are
            # independent chains) on a column sample of the same keyframe, + bit-exact parity with the GPU
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle
            cols = np.random.default_rng(args.seed + 3).choice(Q, min(Q, 3000), replace=False)
            src = [x.view(F, Q)[:, cols].cpu().numpy() for x in (out_tile, out_pal, out_hm, out_vm)]
            t0 = time.perf_counter()
            o = pyoracle.smooth(src[0], src[1], src[2], src[3], np.zeros((F, cols.size), np.uint8), tiles, pals, 0.02)
            tc = time.perf_counter() - t0
            g = [x[:, cols].cpu().numpy() for x in (s_tile, s_pal, s_hm, s_vm, s_sm)]
            smooth["cpu_baseline"] = {"value": round((F - 1) * cols.size / tc / 1e6, 6), "unit": "Msteps/s",
                                      "cores": 1, "kind": "port",
                                      "sample": f"{cols.size} random positions x {F} frames of the same keyframe "
                                                f"(or_smooth, two fp64 DCT descriptors per step, one thread)"}
            smooth["parity_positions"] = int(cols.size)
            smooth["parity_mismatches_vs_cpu"] = int(sum(np.count_nonzero(np.asarray(a) != np.asarray(b))
                                                         for a, b in zip(g, o[:5])))

    # ---- secondary: the Load step's keyframe detection over a whole clip (main.pas:1099-1146) ----
    keyframes = None
    if rank == 0 and not args.no_keyframes:
        from tiler_amd.keyframes import find_keyframes
        tw, th, FC = W // 8, H // 8, args.clip_frames
        g = torch.Generator(device=dev)
        g.manual_seed(args.seed)
        clip = torch.randint(0, 1 << 24, (FC, Q * 64), dtype=torch.int32, device=dev, generator=g)
        corr = np.zeros(FC - 1, np.float64)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        check(lib.tiler_interframe_correlation_dev(vp(clip.data_ptr()), FC, tw, th, corr.ctypes.data_as(vp),
                                                   vp(stream)), "tiler_interframe_correlation_dev")
        _, n_kf = find_keyframes(corr, FC, Q)
        tk = time.perf_counter() - t0
        keyframes = {"value": round((FC - 1) / tk, 2), "unit": "frame pairs/s", "ms": round(tk * 1e3, 3),
                     "keyframes": int(n_kf), "shape": f"{FC} frames {W}x{H} (random bytes, generated in HBM), "
                                                      f"Pearson over 3*{W * H} bytes per pair",
                     "bound": "sequential fp64 chains (the reference's summation order): producer waves compute the terms, one adder lane per frame"}
        if world == 1 and not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle
            ns = min(8, FC - 1)
            sample = clip[:ns + 1].cpu().numpy()
            t0 = time.perf_counter()
            ocorr = pyoracle.interframe_corr_batch(sample, tw, th)
            tc = time.perf_counter() - t0
            keyframes["cpu_baseline"] = {"value": round(ns / tc, 2), "unit": "frame pairs/s", "cores": 1,
                                         "kind": "port", "sample": f"the clip's first {ns} pairs (oracle/load_kf.c; "
                                                                   "the reference runs this loop on one thread)"}
            keyframes["parity_mismatches_vs_cpu"] = int(np.sum(ocorr.view(np.uint64) != corr[:ns].view(np.uint64)))
        del clip

    # ---- secondary: the Dither step per tile (DitherTile, Thomas Knoll, + PrepareTileMirrors) over this step's
    # frames with the keyframe's 128 palettes (FinishDitherTiles main.pas:2482-2544) ----
    dither = None
    if rank == 0 and not args.no_dither:
        from tiler_amd.dither import dither_tiles_dev
        rng_d = np.random.default_rng(args.seed + 7)
        pal_of = rng_d.integers(0, P, QK).astype(np.int32)
        d_pal_of = torch.from_numpy(pal_of).to(dev)
        d_px = torch.empty((QK, 64), dtype=torch.uint8, device=dev)
        d_dhm = torch.empty(QK, dtype=torch.uint8, device=dev)
        d_dvm = torch.empty(QK, dtype=torch.uint8, device=dev)
        call = lambda: dither_tiles_dev(QK, d_rgb.data_ptr(), d_pal_of.data_ptr(), d_pals.data_ptr(), P, 16,  # noqa: E731
                                        d_px.data_ptr(), d_dhm.data_ptr(), d_dvm.data_ptr(), stream)
        call()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        call()
        torch.cuda.synchronize(dev)
        td = time.perf_counter() - t0
        dither = {"value": round(QK / td / 1e6, 4), "unit": "Mtiles/s", "ms": round(td * 1e3, 3),
                  "shape": f"{QK} tiles ({F} frames {W}x{H}), palettes {P} x 16, Thomas Knoll mixing (64 x 16 "
                           f"colour compares per pixel) + luma QuickSort + PrepareTileMirrors"}
        if world == 1 and not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle
            ns = 400
            sample = frames.reshape(-1, 64)[:ns]
            t0 = time.perf_counter()
            opx, ohm, ovm = pyoracle.dither_tiles_tk(sample, pal_of[:ns], pals)
            tc = time.perf_counter() - t0
            gpx = d_px[:ns].cpu().numpy()
            dither["cpu_baseline"] = {"value": round(ns / tc / 1e6, 6), "unit": "Mtiles/s", "cores": 1, "kind": "port",
                                      "sample": f"the first {ns} tiles (oracle/dither_tk.c, no colour cache)"}
            dither["parity_mismatches_vs_cpu"] = int(np.sum(np.any(gpx != opx, axis=1)) +
                                                     np.sum(d_dhm[:ns].cpu().numpy() != ohm) +
                                                     np.sum(d_dvm[:ns].cpu().numpy() != ovm))
        # the non-default branch (chkUseTK off): Yliluoma mixing at the form's default cbxYilMix = 4
        yl_call = lambda: dither_tiles_dev(QK, d_rgb.data_ptr(), d_pal_of.data_ptr(), d_pals.data_ptr(), P, 16,  # noqa: E731
                                           d_px.data_ptr(), d_dhm.data_ptr(), d_dvm.data_ptr(), stream, yliluoma_mix=4)
        yl_call()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        yl_call()
        torch.cuda.synchronize(dev)
        ty = time.perf_counter() - t0
        yl = {"value": round(QK / ty / 1e6, 4), "unit": "Mtiles/s", "ms": round(ty * 1e3, 3),
              "shape": "the same tiles and palettes, Yliluoma mixing (DeviseBestMixingPlanYliluoma's ASM_DBMP form, "
                       "Y2MixedColors 4) + luma QuickSort + PrepareTileMirrors"}
        if world == 1 and not args.no_cpu:
            ns = 400
            t0 = time.perf_counter()
            opx, ohm, ovm = pyoracle.dither_tiles_yl(sample, pal_of[:ns], pals, 4)
            tc = time.perf_counter() - t0
            yl["cpu_baseline"] = {"value": round(ns / tc / 1e6, 6), "unit": "Mtiles/s", "cores": 1, "kind": "port",
                                  "sample": f"the first {ns} tiles (oracle/dither_tk.c or_dither_tiles_yl, no colour cache)"}
            yl["parity_mismatches_vs_cpu"] = int(np.sum(np.any(d_px[:ns].cpu().numpy() != opx, axis=1)) +
                                                 np.sum(d_dhm[:ns].cpu().numpy() != ohm) +
                                                 np.sum(d_dvm[:ns].cpu().numpy() != ovm))
        dither["yliluoma"] = yl
        del d_px, d_dhm, d_dvm, d_pal_of

    # ---- secondary: the Dither step's palette generation over one keyframe (btnDitherClick main.pas:886-907):
    # PrepareDitherTiles (LAB descriptors + k-means, k = 128), QuantizePalette (DLv3) for the 128 palettes,
    # FinishQuantizePalette; frames: a 1080p shot (smooth 16-px blocks + +-2 noise, synth.shot_frames) ----
    palettes_line = None
    if rank == 0 and not args.no_palettes:
        from tiler_amd.palette import generate_palettes
        pf, _ = synth.shot_frames(np.random.default_rng(args.seed + 11), args.palette_frames, W // 8, H // 8,
                                  shot_len=(args.palette_frames, args.palette_frames), noise=2)
        kfs = np.array([0, pf.shape[0]])
        generate_palettes(pf[:1], np.array([0, 1]), P)  # warm-up (allocations, code objects)
        torch.cuda.synchronize(dev)
        lib.tiler_timing_reset()
        lib.tiler_timing_enable(1)
        t0 = time.perf_counter()
        gp, gc, gd, guc = generate_palettes(pf, kfs, P)
        tp = time.perf_counter() - t0
        lib.tiler_timing_enable(0)
        ph = {}
        for name in ("psyv", "kmeans", "kmeans_assign", "kmeans_update", "dl3_table", "dl3_pass1", "dl3_reduce"):
            n = ctypes.c_int(0)
            ms = lib.tiler_timing_get(name.encode(), ctypes.byref(n))
            ph[name] = round(ms, 2)
        nt = pf.shape[0] * Q
        palettes_line = {"value": round(nt / tp / 1e6, 4), "unit": "Mtiles/s", "ms": round(tp * 1e3, 1),
                         "phases_ms": ph, "use_count_max": int(guc.max()),
                         "shape": f"{pf.shape[0]} frames {W}x{H} ({nt} tiles), {P} palettes x 16, DLv3 bpc 7"}
        if world == 1 and not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle
            # bounded sample: DLv3 of the 8 smallest palettes of this keyframe (the GPU's DitheringPalIndex),
            # each restated on one host thread; rate in palettes/s beside the GPU's 128 palettes in its DLv3 time
            order = np.argsort(np.bincount(gd, minlength=P), kind="stable")
            sel = [int(p) for p in order if 0 < np.count_nonzero(gd == p)][:8]
            tiles_all = pf.reshape(-1, 64)
            t0 = time.perf_counter()
            mism = 0
            for p in sel:
                m = gd == p
                op_, ouc, _ = pyoracle.quantize_palettes(tiles_all[m], np.zeros(int(m.sum()), np.int32), 1, threads=1)
                mism += int(not np.array_equal(op_[0], gp[0][p]))
            tc = time.perf_counter() - t0
            dl3_s = (ph["dl3_table"] + ph["dl3_pass1"] + ph["dl3_reduce"]) / 1e3
            palettes_line["cpu_baseline"] = {
                "value": round(len(sel) / tc, 3), "unit": "palettes/s (QuantizePalette, DLv3)", "cores": 1,
                "kind": "port", "sample": f"the {len(sel)} smallest palettes of the keyframe (oracle/palette.c)",
                "gpu_palettes_per_s": round(P / dl3_s, 2) if dl3_s else None}
            palettes_line["parity_palettes"] = len(sel)
            palettes_line["parity_mismatches_vs_cpu"] = mism

    # ---- secondary: the palettes of SEVERAL keyframes in one call, as btnDitherClick runs DoQuantize over every
    # (keyframe, palette) pair at once (main.pas:901): what a clip pays per keyframe when the pairs share the GPU ----
    palettes_clip = None
    if rank == 0 and world == 1 and not args.no_palettes and args.palette_keyframes > 1:
        from tiler_amd.palette import generate_palettes
        nk, fpk = args.palette_keyframes, args.palette_frames
        cf, _ = synth.shot_frames(np.random.default_rng(args.seed + 13), nk * fpk, W // 8, H // 8,
                                  shot_len=(fpk, fpk), noise=2)
        kfs = np.arange(0, nk * fpk + 1, fpk)
        torch.cuda.synchronize(dev)
        lib.tiler_timing_reset()
        lib.tiler_timing_enable(1)
        t0 = time.perf_counter()
        generate_palettes(cf, kfs, P)
        tp = time.perf_counter() - t0
        lib.tiler_timing_enable(0)
        ph = {}
        for name in ("kmeans", "dl3_table", "dl3_pass1", "dl3_reduce"):
            n = ctypes.c_int(0)
            ph[name] = round(lib.tiler_timing_get(name.encode(), ctypes.byref(n)), 2)
        palettes_clip = {"value": round(tp / nk, 4), "unit": "s per keyframe (amortised)", "s": round(tp, 3),
                         "keyframes": nk, "pairs": nk * P, "phases_ms": ph,
                         "shape": f"{nk} keyframes x {fpk} frames {W}x{H}, {P} palettes x 16 each, DLv3 of all "
                                  f"{nk * P} (keyframe, palette) pairs in one pass (k-means per keyframe)"}
        del cf

    # ---- secondary: GlobalTiling K-Modes at C4 (BASELINE.json config 4; bench_globaltiling.py) ----
    gtl = None
    if rank == 0 and not args.no_globaltiling:
        import bench_globaltiling
        ga = bench_globaltiling.parser().parse_args([])
        ga.no_cpu = args.no_cpu or world > 1
        ga.cpu_seconds = min(10.0, args.cpu_seconds)
        gtl = bench_globaltiling.run(ga)

    # ---- secondary: the reference's unmodified per-tile call pattern (main.pas:4027 from every ProcThreadPool worker,
    # main.pas:972) on this keyframe's ONE handle: ann_kdtree_search per query, one thread (latency) and 16 threads
    # (the library coalesces concurrent callers into batches); every answer checked against the batched search ----
    per_call = None
    if rank == 0 and world == 1 and not args.no_per_call:
        per_call = per_call_line(lib, kdt, frames, args.per_call_queries)

    # ---- secondary: the encoder's whole FrameTiling pass over the 1000-frame C3 clip with REAL PrepareFrameTiling
    # candidate sets (bench_encoder.py: PrepareGlobalFT, per keyframe Prepare at Medium quality + FrameTiling + Smooth),
    # items shot-local (16k tiles per keyframe) and from the whole tileset ----
    enc_local = enc_all = None
    if rank == 0 and world == 1 and not args.no_encoder and args.config == "c3":
        import bench_encoder
        for name, item_tiles in (("local", 16384), ("all", 0)):
            ea = bench_encoder.parser().parse_args(["--item-tiles", str(item_tiles)])
            ea.check_kf = -1 if args.no_cpu else 1
            r = bench_encoder.run(ea)
            print(f"[bench] encoder_{name}: {r['value']} Mtiles/s, parity {r.get('parity')}", file=sys.stderr,
                  flush=True)
            r.pop("diag", None)
            if name == "local":
                enc_local = r
            else:
                enc_all = r
            torch.cuda.empty_cache()

    # ---- CPU baseline (rank 0, N=1): the oracle restatement, bounded sample, same workload ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, tiles, thm, tvm, pals, ds, frames, out_tile, out_pal, out_hm, out_vm, out_err)

    if rank == 0:
        res = {
            "metric": METRIC, "value": round(value, 4), "unit": "Mtiles/s", "n_gpus": world, "ranks_seen": ranks_seen,
            "process_group": dist.get_backend() if use_dist else None,
            "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded, SURVEY.md 8(d))",
            "config": {"workload": f"{args.config.upper()}: {W}x{H} 8x8 tiles ({Q} tiles/frame), keyframe of {F} "
                                   f"frames per GPU per step, {TS} tileset x 4 mirrors = {M} candidates (P_eff=1)",
                       "tiles_per_step_per_gpu": QK, "candidates": M, "descriptor": "PsyV Haar 192-d",
                       "parallelism": f"keyframes sharded, {world} GPU(s)"},
            "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels, "search_stats": stats, "out_digest": out_digest,
            "secondary": {"prepare": prep, "smooth": smooth, "keyframes": keyframes, "dither": dither,
                          "palettes": palettes_line, "palettes_clip": palettes_clip, "globaltiling": gtl,
                          "per_tile_calls": per_call,
                          "encoder_local": enc_local, "encoder_all": enc_all},
        }
        print(json.dumps(res))
    kdt.close()
    if use_dist:
        dist.destroy_process_group()


def rank_check() -> None:
    """--rank-check: rendezvous the ranks over gloo (CPU only), all-reduce (rank + 1) and print the world seen."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    seen, total = 1, 1
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([rank + 1], dtype=torch.int64)
        dist.all_reduce(t)
        seen, total = dist.get_world_size(), int(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_seen": seen, "rank_sum": total,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}))


def launch_ranks(n: int) -> int:
    """Start `n` ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in each one's environment, as
    torch.distributed.run would set them; rank r binds GPU r), relay rank 0's stdout and return the worst exit
    status.  The parent never initialises the GPU, so the children are plain child processes, not an exec.
    If a rank fails, the others are stopped (by their own PIDs) so nobody waits at a barrier forever."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = []
    import threading
    reader = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode().splitlines()), daemon=True)
    reader.start()
    codes = [None] * n
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
                if codes[i] not in (None, 0):
                    for q in procs:
                        if q.poll() is None:
                            q.kill()
        time.sleep(0.2)
    reader.join(timeout=30)
    for ln in out0:
        print(ln, flush=True)
    bad = [c for c in codes if c]
    if bad:
        print(f"bench.py: rank exit codes {codes}", file=sys.stderr)
    return (bad[0] if bad[0] > 0 else 128 - bad[0]) if bad else 0


def per_call_line(lib, kdt, frames, nq_conc: int) -> dict:
    """ann_kdtree_search once per query, as DoFrameTiling calls it (main.pas:4023-4027), on the keyframe's handle:
    latency of lone calls, then calls/s with 16 threads calling concurrently on the same handle.  The queries are
    the keyframe's frame tiles' descriptors (fp32, made on the GPU); every answer must equal the batched search's."""
    import ctypes
    import threading
    from tiler_amd.psyv import psyv_batch
    nq = min(nq_conc, frames.reshape(-1, 64).shape[0])
    _, qd = psyv_batch(rgb=frames.reshape(-1, 64)[:nq], flags=2, want64=False, want32=True)
    bi, be = kdt.search_batch(qd)
    ref_i, ref_e = bi.astype(np.int64), be
    err = np.zeros(1, np.float32)
    vp = ctypes.c_void_p
    lat = []
    one = np.zeros(nq, np.int64)
    for i in range(64):  # lone calls: the full per-call path (H2D, search chain, D2H, sync)
        q = np.ascontiguousarray(qd[i])
        t0 = time.perf_counter()
        one[i] = lib.ann_kdtree_search(kdt.handle, q.ctypes.data_as(vp), 0.0, err.ctypes.data_as(vp))
        lat.append(time.perf_counter() - t0)
    threads = 16
    # native callers first (tiler_debug_percall_bench: std::threads inside libANN.so, no interpreter between calls)
    n_idx = np.zeros(nq, np.int32)
    n_err = np.zeros(nq, np.float32)
    wall, lone_us = ctypes.c_double(0), ctypes.c_double(0)
    qc = np.ascontiguousarray(qd[:nq], np.float32)
    n0 = kdt.combine_stats()
    rc = lib.tiler_debug_percall_bench(kdt.handle, qc.ctypes.data_as(vp), nq, 1, threads, n_idx.ctypes.data_as(vp),
                                       n_err.ctypes.data_as(vp), ctypes.byref(wall), ctypes.byref(lone_us))
    n1 = kdt.combine_stats()
    native = None
    if rc == 0:
        nb = (n1["batches"] - n0["batches"])
        native = {"calls_per_s": round(nq / wall.value, 1), "lone_call_us_median": round(lone_us.value, 1),
                  "batches": int(nb), "avg_batch": round((n1["calls"] - n0["calls"]) / max(1, nb), 2),
                  "mismatches_vs_batched": int(np.count_nonzero(n_idx != ref_i) +
                                               np.count_nonzero(n_err.view(np.uint32) != ref_e.view(np.uint32)))}
    got = np.full(nq, -2, np.int64)
    gerr = np.zeros(nq, np.float32)
    c0 = kdt.combine_stats()

    def worker(t):
        e = np.zeros(1, np.float32)
        for i in range(t, nq, threads):
            got[i] = lib.ann_kdtree_search(kdt.handle, qd[i].ctypes.data_as(vp), 0.0, e.ctypes.data_as(vp))
            gerr[i] = e[0]

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    tc = time.perf_counter() - t0
    c1 = kdt.combine_stats()
    batches = c1["batches"] - c0["batches"]
    mism = int(np.count_nonzero(got != ref_i) + np.count_nonzero(gerr.view(np.uint32) != ref_e.view(np.uint32)) +
               np.count_nonzero(one[:64] != ref_i[:64]))
    lat_ms = np.array(lat) * 1e3
    return {"value": native["calls_per_s"] if native else None,
            "unit": "calls/s (16 native threads, one handle)", "native": native,
            "python_threads": {"calls_per_s": round(nq / tc, 1), "note": "16 Python threads via ctypes (GIL between "
                                                                        "calls): harness-bound"},
            "queries": nq,
            "threads": threads, "latency_ms": {"median": round(float(np.median(lat_ms)), 3),
                                               "p90": round(float(np.percentile(lat_ms, 90)), 3)},
            "lone_calls_per_s": round(1e3 / float(np.median(lat_ms)), 1),
            "batches": int(batches), "avg_batch": round(nq / max(1, batches), 2), "max_batch": c1["max_batch"],
            "mismatches_vs_batched": mism,
            "what": "ann_kdtree_search (extern.pas:65) per frame tile on the C3 keyframe handle; concurrent callers "
                    "are coalesced into batches inside libANN.so (ann_api.hip Combiner)"}


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes (profiles/pmc_traffic.json,
    written by profiles/summarize.py from profiles/run_profile.sh on the GPU box; counters cannot be
    collected inside the timed run)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        k = t["kernels"][kernel]
        return int(k["hbm_traffic_bytes"]), f"profiles/pmc_traffic.json ({t['source']})"
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(args, tiles, thm, tvm, pals, ds, frames, out_tile, out_pal, out_hm, out_vm, out_err):
    """The reference's CPU FrameTiling path on the box's host cores, bounded sample of the same keyframe:
    the query descriptor (ComputeTilePsyVisFeatures, fp64) + the ANN 1.1.2 kd-tree search (ANN_KD_STD,
    bucket 1, eps 0: oracle/ann_kdtree.c), timed.  Every sampled query is also the parity check: tile,
    palette, mirror flags and fp32 distance must equal the GPU's bit for bit (the GPU reproduces ANN's
    first-found tie order, tiler_amd/csrc/kdtree.hip); `index_order_would_differ` counts the queries where
    resolving ties to the lowest index instead would have changed the item."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    from benchutil import host_cores
    hc = host_cores()
    threads = args.cpu_threads or hc["usable"]
    P, T = pals.shape[0], tiles.shape[0]
    used = np.zeros((P, T, 4), np.uint8)
    used[ds.pal_of, ds.tile_of, ds.attrs] = 1
    ods, ot, op, oa = pyoracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    t0 = time.perf_counter()
    kd = pyoracle.KDTree(ods)
    build_s = time.perf_counter() - t0
    q0 = frames.reshape(-1, 64)
    g = [t.cpu().numpy() for t in (out_tile, out_pal, out_hm, out_vm, out_err)]
    done, chunk, spent = 0, 8 * threads, 0.0
    mism = dist_mism = 0
    qd_all, ke_all = [], []
    # chunks alternately from the front and the back of the keyframe: the back's queries sit in the last,
    # possibly candidate-split, workgroups of the shortlist launch (orbit_search's mixed split)
    front, back, it = 0, q0.shape[0], 0
    while spent < args.cpu_seconds and front < back:
        if it % 2 == 0:
            sl = slice(front, min(front + chunk, back))
            front = sl.stop
        else:
            sl = slice(max(back - chunk, front), back)
            back = sl.start
        it += 1
        t0 = time.perf_counter()
        qd = pyoracle.psyv_batch(sl.stop - sl.start, rgb=q0[sl], flags=2).astype(np.float32)
        ki, ke = kd.search_batch(qd, threads=threads)
        spent += time.perf_counter() - t0
        print(f"[bench] cpu baseline: {done + sl.stop - sl.start} queries, {spent:.1f} s", file=sys.stderr, flush=True)
        dist_mism += int(np.count_nonzero(ke.view(np.uint32) != g[4][sl].view(np.uint32)))
        same = (ot[ki] == g[0][sl]) & (op[ki] == g[1][sl]) & ((oa[ki] & 1) == g[2][sl]) & ((oa[ki] >> 1) == g[3][sl])
        mism += int(np.count_nonzero(~same))
        qd_all.append(qd)
        ke_all.append(ki)
        done += sl.stop - sl.start
    visited = kd.visited / max(done, 1)
    kd.close()
    # the same sample under the lowest-index rule (exhaustive scan): how often the tie rule decides the item
    qd_all = np.concatenate(qd_all)
    ki_all = np.concatenate(ke_all)
    li, _ = pyoracle.nn_batch(ods, qd_all, threads=threads)
    tie_decided = int(np.count_nonzero((ot[li] != ot[ki_all]) | (oa[li] != oa[ki_all]) | (op[li] != op[ki_all])))
    return {"value": round(done / spent / 1e6, 6), "unit": "Mtiles/s", "cores": threads, "kind": "port",
            "host_cores": hc,
            "sample": f"{done} query tiles of the keyframe (first {front} and last {q0.shape[0] - back}) vs the full "
                      f"{ods.shape[0]}-candidate set: fp64 "
                      f"descriptor + ANN 1.1.2 kd-tree (ANN_KD_STD, bucket 1, eps 0; oracle/ann_kdtree.c; "
                      f"{visited:.0f} leaves visited per query, tree build {build_s:.1f} s untimed), {threads} threads",
            "parity_queries": done, "parity_mismatches_vs_gpu": mism, "dist_mismatches_vs_gpu": dist_mism,
            "index_order_would_differ": tie_decided}


if __name__ == "__main__":
    main()

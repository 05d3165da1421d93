"""Test worker (its own process: tiler_init(TILER_ALL_DEVICES) must be the library's first binding, and the pytest
process is already bound to device 0).  Run by tests/test_gpu_multidevice.py; prints one JSON line of findings.

The reference encoder is ONE process (main.pas:972): every keyframe's handle is made by ann_kdtree_create from host
rows (main.pas:3961) and searched per tile from pool threads (main.pas:4027); PrepareFrameTiling's UseOne searches the
global 64-d dataset (main.pas:3779, 3830).  Here all of that runs with every visible device bound: the handles are
placed by the library's rule, the calls are checked bit for bit against the restated ANN search, and the replication
path (copy of a handle's index on the device of a device-buffer call) is forced on the handle's own device so that
it runs on a one-GPU box too.
"""
import ctypes
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

torch.cuda.init()
import pyoracle  # noqa: E402
import tiler_amd  # noqa: E402
from tiler_amd import frame_tiling as ft  # noqa: E402
from tiler_amd import synth  # noqa: E402
from tiler_amd._lib import check  # noqa: E402

THREADS = 16


def threads(fn, n):
    errs = []

    def w(t):
        try:
            for i in range(t, n, THREADS):
                fn(i)
        except Exception as e:
            errs.append(e)

    ths = [threading.Thread(target=w, args=(t,)) for t in range(THREADS)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]


def main():
    out = {}
    lib = tiler_amd.load()
    assert lib.tiler_init(-1) == 0, tiler_amd.last_error()
    ndev = lib.tiler_device_count()
    out["devices"] = ndev
    assert lib.tiler_init(0) == -1  # bound to all: a single-device rebinding is refused
    rng = np.random.default_rng(77)
    pals = synth.palettes(rng, 8)

    # ---- keyframe handles from host rows (ann_kdtree_create, main.pas:3961), placed by the library's rule ----
    sizes = [1500, 2500, 1200, 3000]
    dss, kdts, qs, tilesets = [], [], [], []
    for n in sizes:
        tiles, thm, tvm = synth.tileset(rng, n)
        used = synth.used_one_palette(rng.integers(0, 8, n).astype(np.int32), 8)
        ods, ot, op, oa = pyoracle.build_ft_dataset(used, tiles, thm, tvm, pals)
        dss.append((ods, ot, op, oa))
        tilesets.append((tiles, thm, tvm))
        kdts.append(tiler_amd.KDTree(ods))
        qs.append(pyoracle.psyv_batch(600, rgb=synth.frame_tiles(rng, 600), flags=2).astype(np.float32))
    bytes_ = np.array([d[0].size * 4 for d in dss], np.int64)
    plan = np.zeros(len(sizes), np.int32)
    assert lib.tiler_placement_plan(ndev, bytes_.ctypes.data_as(ctypes.c_void_p), len(sizes),
                                    plan.ctypes.data_as(ctypes.c_void_p)) == 0
    out["placement"] = [k.device() for k in kdts]
    out["plan"] = plan.tolist()

    # ---- per-tile calls from 16 threads spread over the keyframes' handles (the concurrent DoFrm pattern) ----
    nq = sum(q.shape[0] for q in qs)
    which = np.concatenate([np.full(q.shape[0], h) for h, q in enumerate(qs)])
    row = np.concatenate([np.arange(q.shape[0]) for q in qs])
    gi = np.full(nq, -7, np.int64)
    ge = np.zeros(nq, np.float32)

    def one(i):
        gi[i], ge[i] = kdts[which[i]].search(qs[which[i]][row[i]])
    threads(one, nq)
    mism = 0
    for h, (ods, *_r) in enumerate(dss):
        okd = pyoracle.KDTree(ods)
        oi, oe = okd.search_batch(qs[h])
        okd.close()
        sel = which == h
        mism += int(np.count_nonzero(gi[sel] != oi) + np.count_nonzero(ge[sel].view(np.uint32) != oe.view(np.uint32)))
    out["per_tile_mismatches"] = mism
    out["per_tile_queries"] = nq

    # ---- the global 64-d dataset (PrepareGlobalFT main.pas:3763-3779) with k = 8 per item from 16 threads ----
    gtiles, gthm, gtvm = synth.tileset(rng, 700)
    gds = ft.prepare_global_ft(gtiles)
    items = rng.integers(0, gtiles.shape[0], 900)
    gq = gtiles[items].astype(np.float32)
    k8i = np.zeros((gq.shape[0], 8), np.int32)
    k8e = np.zeros((gq.shape[0], 8), np.float32)

    def one8(i):
        k8i[i], k8e[i] = gds.kdt.search_multi(gq[i], 8)
    threads(one8, gq.shape[0])
    ogds, ogt, oga = pyoracle.prepare_global_ds(gtiles)
    okd = pyoracle.KDTree(ogds)
    oi8, oe8 = okd.search_batch(gq, k=8)
    okd.close()
    out["k8_mismatches"] = int(np.count_nonzero(k8i != oi8) + np.count_nonzero(k8e.view(np.uint32) != oe8.view(np.uint32)))

    # ---- the device-buffer entry points on the global handle and on a keyframe: without copies, then with copies ----
    dev = torch.device("cuda", 0)
    P, T = 8, gtiles.shape[0]
    gpals = synth.palettes(rng, P)
    cent = synth.palette_centroids(gpals)
    near = ft.near_palettes(cent)
    it_t = rng.integers(0, T, 3000).astype(np.int32)
    it_p = rng.integers(0, P, 3000).astype(np.int32)
    d = {k: torch.from_numpy(np.ascontiguousarray(a)).to(dev) for k, a in
         (("t", it_t), ("p", it_p), ("tiles", gtiles), ("thm", gthm), ("tvm", gtvm), ("pals", gpals))}
    frames = synth.frame_tiles(rng, 1200)
    d_rgb = torch.from_numpy(frames.reshape(-1, 64)).to(dev)

    def prepare_and_tile(tag):
        kt, info = ft.prepare_frame_tiling_dev(gds, d["t"].data_ptr(), d["p"].data_ptr(), it_t.size,
                                               d["tiles"].data_ptr(), d["thm"].data_ptr(), d["tvm"].data_ptr(), T,
                                               d["pals"].data_ptr(), P, ft.FT_MEDIUM, near)
        torch.cuda.synchronize(dev)
        maps = kt.maps()
        Q = frames.shape[0]
        o = [torch.empty(Q, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.uint8, torch.uint8,
                                                            torch.float32)]
        vp = ctypes.c_void_p
        check(lib.tiler_frame_tiling_dev(kt.handle, vp(d_rgb.data_ptr()), Q, 1, -1,
                                                   *[vp(x.data_ptr()) for x in o], None), "tiler_frame_tiling_dev")
        torch.cuda.synchronize(dev)
        host = ft.KeyframeTiler.__new__(ft.KeyframeTiler)  # the host entry point runs on the handle itself
        host.kdt, host.use_wavelets, host.gamma = kt, True, -1
        h = host.do_frame_tiling(frames)
        kt.close()
        return info, maps, [x.cpu().numpy() for x in o], list(h)

    info0, maps0, dev0, host0 = prepare_and_tile("direct")
    lib.tiler_debug_force_replicas(1)
    kdts[0].replicate(-1)
    # a search through device buffers on a handle with a copy runs on the copy
    q0 = torch.from_numpy(qs[0]).to(dev)
    di = torch.empty(qs[0].shape[0], dtype=torch.int32, device=dev)
    de = torch.empty(qs[0].shape[0], dtype=torch.float32, device=dev)
    kdts[0].search_batch_dev(q0.data_ptr(), qs[0].shape[0], 1, di.data_ptr(), de.data_ptr())
    torch.cuda.synchronize(dev)
    okd = pyoracle.KDTree(dss[0][0])
    oi, oe = okd.search_batch(qs[0])
    okd.close()
    out["replica_search_mismatches"] = int(np.count_nonzero(di.cpu().numpy() != oi) +
                                           np.count_nonzero(de.cpu().numpy().view(np.uint32) != oe.view(np.uint32)))
    info1, maps1, dev1, host1 = prepare_and_tile("replicated global dataset")  # gds's copy serves the k = 8 search
    out["prepare_same"] = bool(info0 == info1 and all(np.array_equal(a, b) for a, b in zip(maps0, maps1)))
    out["ft_dev_same"] = bool(all(np.array_equal(a, b) for a, b in zip(dev0, dev1)))
    out["ft_host_same"] = bool(all(np.array_equal(a, b) for a, b in zip(host0, host1)) and
                               all(np.array_equal(a, b) for a, b in zip(dev0, host0)))
    # maps set after a copy exists reach the copy: a keyframe handle with maps, copied, then FrameTiling through it
    tiles, thm, tvm = tilesets[3]
    ods, ot, op, oa = dss[3]
    kt = kdts[3]
    kt.replicate(-1)
    vp = ctypes.c_void_p
    check(lib.tiler_ft_set_maps(kt.handle, ot.ctypes.data_as(vp), op.ctypes.data_as(vp),
                                          oa.ctypes.data_as(vp)), "tiler_ft_set_maps")
    Q = frames.shape[0]
    o = [torch.empty(Q, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.uint8, torch.uint8,
                                                        torch.float32)]
    check(lib.tiler_frame_tiling_dev(kt.handle, vp(d_rgb.data_ptr()), Q, 1, -1,
                                               *[vp(x.data_ptr()) for x in o], None), "tiler_frame_tiling_dev")
    torch.cuda.synchronize(dev)
    ref = pyoracle.frame_tiling(frames, ods, ot, op, oa)
    got = [x.cpu().numpy() for x in o]
    out["replica_ft_mismatches"] = int(sum(np.count_nonzero(a != b) for a, b in zip(got[:4], ref[:4])) +
                                       np.count_nonzero(got[4].view(np.uint32) != ref[4].view(np.uint32)))
    # a device create on a caller's stream that is still busy, copied at once with no host sync in between: the copy
    # must wait for the rows copy and index build queued on that stream (replica_of's ready_ev)
    ods1 = dss[1][0]
    src = torch.from_numpy(ods1).to(dev)
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        busy = torch.rand(4096, 4096, device=dev)
        for _ in range(24):
            busy = busy @ busy * (1.0 / 4096)
        rows_late = src * 1.0  # the dataset is written on `side` only after the busy work
    kt1 = tiler_amd.KDTree(dev_ptr=rows_late.data_ptr(), n=ods1.shape[0], dd=ods1.shape[1], stream=side.cuda_stream)
    kt1.replicate(-1)
    q1 = torch.from_numpy(qs[1]).to(dev)
    di1 = torch.empty(qs[1].shape[0], dtype=torch.int32, device=dev)
    de1 = torch.empty(qs[1].shape[0], dtype=torch.float32, device=dev)
    kt1.search_batch_dev(q1.data_ptr(), qs[1].shape[0], 1, di1.data_ptr(), de1.data_ptr())
    torch.cuda.synchronize(dev)
    okd = pyoracle.KDTree(ods1)
    oi1, oe1 = okd.search_batch(qs[1])
    okd.close()
    out["stream_replica_mismatches"] = int(np.count_nonzero(di1.cpu().numpy() != oi1) +
                                           np.count_nonzero(de1.cpu().numpy().view(np.uint32) != oe1.view(np.uint32)))
    kt1.close()
    del busy, rows_late
    lib.tiler_debug_force_replicas(0)
    for k in kdts:
        k.close()
    gds.kdt.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

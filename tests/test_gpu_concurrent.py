"""The reference's unmodified call pattern through the C-ABI (SURVEY.md 8(b) threading).

DoFrameTiling calls ann_kdtree_search ONCE PER TILE (main.pas:4027) from every ProcThreadPool worker on the
keyframe's one KDT handle (main.pas:972), and PrepareFrameTiling's UseOne calls ann_kdtree_search_multi (k = 8) once
per item on FGlobalDS.KDT (main.pas:3830).  Here 16 host threads do exactly that on ONE handle through ctypes (which
releases the GIL, so the calls really overlap inside libANN.so), and every answer must equal the restated ANN 1.1.2
search (oracle/ann_kdtree.c) bit for bit: index, fp32 distance, and for k = 8 the whole ascending list.  The library
coalesces such callers into batches (ann_api.hip, Combiner); the counters show that it did.
"""
import threading

import numpy as np
import pytest

from tiler_amd import synth

pytestmark = pytest.mark.gpu

THREADS = 16


def _run_threads(fn, n_items):
    """fn(i) for i in range(n_items), spread over THREADS threads (each walks its own stride, like a pool's workers)."""
    errors = []

    def worker(t):
        try:
            for i in range(t, n_items, THREADS):
                fn(i)
        except Exception as e:  # surfaced in the main thread
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[0]


def test_concurrent_per_tile_search_one_handle(gpu, oracle):
    """ann_kdtree_search per frame tile, 16 threads, one keyframe handle (mirror-orbit dataset, ANN tie order)."""
    rng = np.random.default_rng(41)
    tiles, thm, tvm = synth.tileset(rng, 3000)
    pals = synth.palettes(rng, 8)
    used = synth.used_one_palette(rng.integers(0, 8, 3000).astype(np.int32), 8)
    ods, *_ = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    nq = 2048
    q = oracle.psyv_batch(nq, rgb=synth.frame_tiles(rng, nq), flags=2).astype(np.float32)
    gi = np.full(nq, -7, np.int64)
    ge = np.zeros(nq, np.float32)
    with gpu.KDTree(ods) as kdt:
        def one(i):
            gi[i], ge[i] = kdt.search(q[i])
        _run_threads(one, nq)
        cs = kdt.combine_stats()
        bi, be = kdt.search_batch(q)  # the batched form on the same handle
    okd = oracle.KDTree(ods)
    oi, oe = okd.search_batch(q)
    okd.close()
    assert np.array_equal(ge.view(np.uint32), oe.view(np.uint32))
    assert np.array_equal(gi, oi)
    assert np.array_equal(bi, oi) and np.array_equal(be.view(np.uint32), oe.view(np.uint32))
    assert cs["calls"] == nq
    assert cs["batches"] < nq  # callers were coalesced (a batch held more than one query)
    assert cs["max_batch"] > 1


def test_concurrent_search_multi_k8_one_handle(gpu, oracle):
    """ann_kdtree_search_multi (cnt = 8) per item, 16 threads, on the PrepareGlobalFT handle (64-d palette-index
    rows of every tile in 4 orientations, main.pas:3763-3779); interleaved with k = 1 calls on the same handle, so the
    coalescer must keep batches of different k apart."""
    rng = np.random.default_rng(42)
    tiles, _, _ = synth.tileset(rng, 2500)
    gds, _, _ = oracle.prepare_global_ds(tiles)
    items = rng.integers(0, tiles.shape[0], 1500)
    q = tiles[items].astype(np.float32)
    gi = np.zeros((q.shape[0], 8), np.int32)
    ge = np.zeros((q.shape[0], 8), np.float32)
    g1 = np.zeros(q.shape[0], np.int64)
    with gpu.KDTree(gds) as kdt:
        def one(i):
            gi[i], ge[i] = kdt.search_multi(q[i], 8)
            if i % 3 == 0:
                g1[i], _ = kdt.search(q[i])
        _run_threads(one, q.shape[0])
        cs = kdt.combine_stats()
    okd = oracle.KDTree(gds)
    oi, oe = okd.search_batch(q, k=8)
    okd.close()
    assert np.array_equal(ge.view(np.uint32), oe.view(np.uint32))
    assert np.array_equal(gi, oi)
    sel = np.arange(0, q.shape[0], 3)
    assert np.array_equal(g1[sel], oi[sel, 0])
    assert cs["calls"] == q.shape[0] + sel.size and cs["batches"] < cs["calls"]


def test_concurrent_errors_reach_every_caller(gpu):
    """A bad call (k out of range) fails for its caller only; concurrent good calls still succeed."""
    data = np.random.default_rng(43).normal(0, 1, (500, 192)).astype(np.float32)
    q = data[:64] + 0.01
    out = np.zeros(64, np.int64)
    with gpu.KDTree(data) as kdt:
        def one(i):
            out[i], _ = kdt.search(q[i])
            if i % 16 == 0:
                with pytest.raises(gpu.TilerError):
                    kdt.search_multi(q[i], 40)
        _run_threads(one, 64)
    assert np.array_equal(out, np.arange(64))


def test_native_percall_harness_exact(gpu, oracle):
    """tiler_debug_percall_bench: the per-call pattern from 16 native threads (no interpreter between calls), k = 1 on
    a keyframe handle and k = 8 on the global 64-d handle; every answer equals the restated ANN search."""
    import ctypes
    vp = ctypes.c_void_p
    lib = gpu.load()
    rng = np.random.default_rng(44)
    tiles, thm, tvm = synth.tileset(rng, 2000)
    pals = synth.palettes(rng, 8)
    used = synth.used_one_palette(rng.integers(0, 8, 2000).astype(np.int32), 8)
    ods, *_ = oracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    q1 = oracle.psyv_batch(3000, rgb=synth.frame_tiles(rng, 3000), flags=2).astype(np.float32)
    gds, _, _ = oracle.prepare_global_ds(tiles)
    q8 = tiles[rng.integers(0, 2000, 1000)].astype(np.float32)
    for data, q, k in ((ods, q1, 1), (gds, q8, 8)):
        idx = np.full((q.shape[0], k), -7, np.int32)
        err = np.zeros((q.shape[0], k), np.float32)
        wall, lone = ctypes.c_double(0), ctypes.c_double(0)
        with gpu.KDTree(data) as kdt:
            rc = lib.tiler_debug_percall_bench(kdt.handle, q.ctypes.data_as(vp), q.shape[0], k, THREADS,
                                               idx.ctypes.data_as(vp), err.ctypes.data_as(vp), ctypes.byref(wall),
                                               ctypes.byref(lone))
            assert rc == 0, gpu.last_error()
            cs = kdt.combine_stats()
        okd = oracle.KDTree(data)
        oi, oe = okd.search_batch(q, k=k)
        okd.close()
        oi, oe = oi.reshape(-1, k), oe.reshape(-1, k)
        assert np.array_equal(idx, oi) and np.array_equal(err.view(np.uint32), oe.view(np.uint32)), k
        assert cs["calls"] == q.shape[0] + min(64, q.shape[0]) and cs["batches"] < cs["calls"]
        print(f"k={k}: {q.shape[0] / wall.value:.0f} calls/s on {THREADS} native threads, lone {lone.value:.1f} us, "
              f"avg batch {cs['calls'] / cs['batches']:.1f}")

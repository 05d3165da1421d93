"""world_size-2 gloo tests of the sharded path on CPU (tiler_amd.dist): keyframe / palette-bin
plans, the tileset broadcast, the K-Modes merge map all-reduce (MAX), the UseCount all-reduce (SUM) and the
tilemap reduce onto one rank give the single-process result, with fixed-layout tensors only.  The per-unit
compute is the CPU oracle here (test-only stand-in for the GPU kernels, which need a device)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tiler_amd import dist as tdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_lpt_plan_balanced_and_complete():
    plan = tdist.plan_keyframes([24, 24, 10, 24, 5, 24, 24, 3], 32400, 4)
    flat = sorted(u for r in plan for u in r)
    assert flat == list(range(8))
    loads = [sum([24, 24, 10, 24, 5, 24, 24, 3][u] for u in r) for r in plan]
    assert max(loads) - min(loads) <= 24
    assert tdist.plan_bins([100, 5, 50, 0], [10, 1, 7, 0], 2) == tdist.plan_bins([100, 5, 50, 0], [10, 1, 7, 0], 2)


def test_no_pickled_collectives_in_product():
    """The product's multi-GPU path exchanges fixed-layout tensors only (no *_object collectives)."""
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tiler_amd")
    for f in os.listdir(root):
        if f.endswith(".py"):
            txt = open(os.path.join(root, f)).read()
            assert "_object(" not in txt, f


KF_FRAMES = [3, 2, 4]
Q = 20


def _kf_frames(u):
    from tiler_amd import synth
    return synth.keyframe_frames(np.random.default_rng(100 + u), KF_FRAMES[u], Q)


def _setup(pyoracle, synth):
    T, P = 300, 4
    rng = np.random.default_rng(5)
    tiles, thm, tvm = synth.tileset(rng, T)
    pals = synth.palettes(np.random.default_rng(6), P)
    tile_pal = np.random.default_rng(7).integers(0, P, T).astype(np.int32)
    ods, ot, op, oa = pyoracle.build_ft_dataset(synth.used_one_palette(tile_pal, P), tiles, thm, tvm, pals)
    return tiles, thm, tvm, ods, ot, op, oa


def _oracle_kmodes_results(pyoracle, plan, bins):
    """DoKModes per bin on the CPU restatement: labels, medoid (GetMinMatchingDissim over the members, ties to the
    last), member counts -- the shape gt.kmodes_bins returns."""
    out = {}
    for p in bins:
        X = plan.lines[plan.bins[p]]
        k = int(plan.k_per_bin[p])
        labels, cent, _, _ = pyoracle.kmodes(X, k, plan.starts[p])
        medoid = np.full(k, -1, np.int32)
        counts = np.bincount(labels, minlength=k).astype(np.int32)
        for j in range(k):
            mem = np.nonzero(labels == j)[0]
            if mem.size:
                i, _ = pyoracle.km_get_min(X[mem], cent[j])
                medoid[j] = mem[i]
        out[p] = (labels, medoid, counts)
    return out


def _gt_inputs():
    from tiler_amd import synth
    rng = np.random.default_rng(9)
    T, P = 900, 5
    tiles = rng.integers(0, 16, (T, 64)).astype(np.uint8)
    tiles[300:600] = tiles[rng.integers(0, 300, 300)]  # duplicates and near-duplicates cluster
    dith = rng.integers(0, P, T).astype(np.int32)
    return tiles, dith, P, synth


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist

    import pyoracle
    from tiler_amd import dist as td
    from tiler_amd import global_tiling as gt
    from tiler_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # 1. tileset broadcast
    tiles, thm, tvm, ods, ot, op, oa = _setup(pyoracle, synth)
    T = tiles.shape[0]
    packed = np.concatenate([tiles.reshape(-1), thm, tvm]).astype(np.int32) if rank == 0 else None
    packed = td.broadcast_array(packed, (T * 64 + 2 * T,), np.int32)
    assert np.array_equal(packed[:T * 64].astype(np.uint8).reshape(T, 64), tiles)
    # 2. GlobalTiling: this rank's palette bins -> merge map -> all-reduce MAX
    gtiles, dith, P, _ = _gt_inputs()
    plan = gt.plan_global_tiling(gtiles, dith, P, desired=200)
    costs = [plan.bins[p].size * max(1, int(plan.k_per_bin[p])) for p in plan.run]
    mine = [plan.run[u] for u in td.lpt_assign(costs, world)[rank]]
    local = gt.kmodes_merge_map(plan, _oracle_kmodes_results(pyoracle, plan, mine), gtiles.shape[0])
    merge_to = td.allreduce(local, "max")
    # 3. FrameTiling: this rank's keyframes -> UseCount all-reduce, tilemaps reduced onto rank 0
    F = sum(KF_FRAMES)
    starts = np.concatenate([[0], np.cumsum(KF_FRAMES)])
    tm = np.zeros((F, Q, 2), np.int32)
    uc = np.zeros(T, np.int64)
    for u in td.plan_keyframes(KF_FRAMES, Q, world)[rank]:
        res = pyoracle.frame_tiling(_kf_frames(u).reshape(-1, 64), ods, ot, op, oa, threads=1)
        tm[starts[u]:starts[u + 1], :, 0] = res[0].reshape(-1, Q)
        tm[starts[u]:starts[u + 1], :, 1] = (res[1] | (res[2].astype(np.int32) << 16) |
                                              (res[3].astype(np.int32) << 17)).reshape(-1, Q)
        np.add.at(uc, res[0], 1)
    uc = td.allreduce(uc, "sum")
    # tilemaps onto rank 0 per keyframe (variable-size units, one buffer per sending rank)
    plan = td.plan_keyframes(KF_FRAMES, Q, world)
    owner = [r for u in range(len(KF_FRAMES)) for r in range(world) if u in plan[r]]
    parts = {u: tm[starts[u]:starts[u + 1]].tobytes() for u in plan[rank]}
    units = td.gather_units(parts, owner, 0)
    assert (units is None) == (rank != 0)
    if rank == 0:
        full = np.concatenate([np.frombuffer(b, np.int32).reshape(-1, Q, 2) for b in units])
        np.savez(out_path, merge_to=merge_to, uc=uc, tm=full)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_steps_match_single_process(tmp_path):
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    import pyoracle
    from tiler_amd import global_tiling as gt
    from tiler_amd import synth
    # merge map: the single process over every bin
    gtiles, dith, P, _ = _gt_inputs()
    plan = gt.plan_global_tiling(gtiles, dith, P, desired=200)
    want = gt.kmodes_merge_map(plan, _oracle_kmodes_results(pyoracle, plan, plan.run), gtiles.shape[0])
    assert np.array_equal(got["merge_to"], want) and (want >= 0).sum() > 0
    pp, act, uc_g, mi = gt.apply_merge_map(got["merge_to"], gtiles, None, None)
    assert act.sum() == gtiles.shape[0] - (want >= 0).sum()
    # FrameTiling tilemaps + UseCount
    tiles, thm, tvm, ods, ot, op, oa = _setup(pyoracle, synth)
    uc = np.zeros(tiles.shape[0], np.int64)
    starts = np.concatenate([[0], np.cumsum(KF_FRAMES)])
    for u in range(len(KF_FRAMES)):
        res = pyoracle.frame_tiling(_kf_frames(u).reshape(-1, 64), ods, ot, op, oa, threads=1)
        blk = got["tm"][starts[u]:starts[u + 1]]
        assert np.array_equal(blk[..., 0].ravel(), res[0])
        assert np.array_equal(blk[..., 1].ravel() & 0xFFFF, res[1])
        assert np.array_equal((blk[..., 1].ravel() >> 16) & 1, res[2])
        assert np.array_equal((blk[..., 1].ravel() >> 17) & 1, res[3])
        np.add.at(uc, res[0], 1)
    assert np.array_equal(got["uc"], uc)


def _save_worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist

    from tiler_amd import synth
    from tiler_amd.encoder import DistributedEncoder

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    v = synth.video(71, 64, 48, kf_frames=(3, 2, 4, 1), n_palettes=4)
    e = DistributedEncoder(v, device=-1)  # host-side only: SaveStream's collective path
    own = sorted(e.plan[rank])
    n_own = sum(int(v.kf_start[k + 1] - v.kf_start[k]) for k in own)
    # a rank holds only its own keyframes' frames and tilemaps
    assert e.kfs == own and e.frames == n_own and e.frame_rgb.shape[0] == n_own and e.tile.shape == (n_own, 48)
    assert np.array_equal(e.frame_rgb, v.frame_rgb[e.frame_idx])
    rng = np.random.default_rng(3)
    sm_full = {"tile": rng.integers(0, e.palpix.shape[0], (v.frames, 48)), "pal": rng.integers(0, 4, (v.frames, 48)),
               "hm": rng.integers(0, 2, (v.frames, 48)).astype(np.uint8),
               "vm": rng.integers(0, 2, (v.frames, 48)).astype(np.uint8),
               "smoothed": (rng.random((v.frames, 48)) < 0.3).astype(np.uint8)}
    e.sm = {k: a[e.frame_idx] for k, a in sm_full.items()}
    data = e.save_stream(64, 48, 24.0)
    assert (data is None) == (rank != 0)
    if rank == 0:
        np.save(out_path, np.frombuffer(data, np.uint8))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_distributed_save_stream_bytes_and_per_rank_memory(tmp_path):
    """SaveStream sharded: each of 2 gloo ranks holds only its keyframes' frames and tilemaps,
    writes and compresses its own keyframe streams, and rank 0 assembles a .gtm byte-identical to the single-process
    writer over the same SmoothedTileMaps (no dense whole-clip tilemap collective)."""
    from tiler_amd import synth
    from tiler_amd.encoder import Encoder
    out = str(tmp_path / "g.npy")
    mp.spawn(_save_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    v = synth.video(71, 64, 48, kf_frames=(3, 2, 4, 1), n_palettes=4)
    e = Encoder(v)
    rng = np.random.default_rng(3)
    e.sm = {"tile": rng.integers(0, e.palpix.shape[0], (v.frames, 48)), "pal": rng.integers(0, 4, (v.frames, 48)),
            "hm": rng.integers(0, 2, (v.frames, 48)).astype(np.uint8),
            "vm": rng.integers(0, 2, (v.frames, 48)).astype(np.uint8),
            "smoothed": (rng.random((v.frames, 48)) < 0.3).astype(np.uint8)}
    assert np.load(out).tobytes() == e.save_stream(64, 48, 24.0)

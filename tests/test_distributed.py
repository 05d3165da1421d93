"""world_size-2 gloo tests of the sharded path on CPU: keyframe / palette-bin plans, tileset broadcast,
tilemap gather and the UseCount all-reduce give the single-process result.  The per-unit compute is the
CPU oracle here (test-only stand-in for the GPU kernels, which need a device)."""
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


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist

    import pyoracle
    from tiler_amd import dist as td
    from tiler_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T, P = 300, 4
    if rank == 0:
        rng = np.random.default_rng(5)
        tiles, thm, tvm = synth.tileset(rng, T)
        packed = np.concatenate([tiles.reshape(-1), thm, tvm]).astype(np.int32)
    else:
        packed = None
    packed = td.broadcast_array(packed, (T * 64 + 2 * T,), np.int32)
    tiles = packed[:T * 64].astype(np.uint8).reshape(T, 64)
    thm = packed[T * 64:T * 64 + T].astype(np.uint8)
    tvm = packed[T * 64 + T:].astype(np.uint8)
    pals = synth.palettes(np.random.default_rng(6), P)
    tile_pal = np.random.default_rng(7).integers(0, P, T).astype(np.int32)
    used = synth.used_one_palette(tile_pal, P)
    ods, ot, op, oa = pyoracle.build_ft_dataset(used, tiles, thm, tvm, pals)
    kf_frames = [3, 2, 4]

    def tile_kf(u):
        fr = synth.keyframe_frames(np.random.default_rng(100 + u), kf_frames[u], 20)
        res = pyoracle.frame_tiling(fr.reshape(-1, 64), ods, ot, op, oa, threads=1)
        return {"tile": res[0], "pal": res[1], "hm": res[2], "vm": res[3], "err": res[4]}

    res = td.run_sharded(3, [f * 20 for f in kf_frames], tile_kf)
    uc = np.zeros(T, np.int64)
    plan = td.plan_keyframes(kf_frames, 20, world)
    for u in plan[rank]:
        np.add.at(uc, res[u]["tile"], 1)
    uc = td.allreduce_sum(uc)
    if rank == 0:
        np.savez(out_path, **{f"{u}_{k}": v for u in res for k, v in res[u].items()}, uc=uc)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_frame_tiling_matches_single_process(tmp_path):
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    # single-process reference
    import pyoracle
    from tiler_amd import synth
    rng = np.random.default_rng(5)
    tiles, thm, tvm = synth.tileset(rng, 300)
    pals = synth.palettes(np.random.default_rng(6), 4)
    tile_pal = np.random.default_rng(7).integers(0, 4, 300).astype(np.int32)
    ods, ot, op, oa = pyoracle.build_ft_dataset(synth.used_one_palette(tile_pal, 4), tiles, thm, tvm, pals)
    uc = np.zeros(300, np.int64)
    for u, f in enumerate([3, 2, 4]):
        fr = synth.keyframe_frames(np.random.default_rng(100 + u), f, 20)
        res = pyoracle.frame_tiling(fr.reshape(-1, 64), ods, ot, op, oa, threads=1)
        assert np.array_equal(got[f"{u}_tile"], res[0]) and np.array_equal(got[f"{u}_err"], res[4])
        np.add.at(uc, res[0], 1)
    assert np.array_equal(got["uc"], uc)

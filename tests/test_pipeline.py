"""End-to-end chain: MakeUnique -> GlobalTiling -> FrameTiling -> Reindex -> Smooth
(btnRunAllClick main.pas:1232-1272) through tiler_amd.encoder (GPU via libANN.so) against the same chain
composed from the CPU restatement, compared after every step: tileset, Active/UseCount, every TileMap
and SmoothedTileMap item bit-exact.  Input: synth.video at C1 (320x240), two keyframes of 3 frames."""
import numpy as np
import pytest

from tiler_amd import synth
from tiler_amd.frame_tiling import FT_FAST, FT_MEDIUM, FT_SLOW


def test_make_unique_step_matches_oracle(oracle):
    """btnDoMakeUniqueClick (host-only step: chunks of FTileMapSize*25 tiles) on the chain's input."""
    from tiler_amd.encoder import Encoder
    v = synth.video(50, 160, 120, kf_frames=(30,), n_palettes=4)
    o = _OracleChain(v)
    T0, Q = o.palpix.shape[0], v.tiles_per_frame
    for first in range(0, T0, Q * 25):
        o.unique(oracle, first, min(Q * 25, T0 - first))
    e = Encoder(v)
    e.do_make_unique()
    assert np.array_equal(e.active, o.active) and np.array_equal(e.tile, o.tile)
    assert np.array_equal(e.palpix, o.palpix) and np.array_equal(e.use_count, o.uc)
    assert 0 < e.active.sum() < e.active.size and T0 > Q * 25  # merged, and more than one chunk


class _OracleChain:
    """The same steps written directly on the oracle (tests only)."""

    def __init__(self, v):
        F, Q = v.frames, v.tiles_per_frame
        self.v = v
        self.palpix = v.palpix.copy()
        self.thm, self.tvm, self.dith = v.thm.copy(), v.tvm.copy(), v.dith_pal.copy()
        self.active = np.ones(F * Q, np.uint8)
        self.uc = np.ones(F * Q, np.int32)
        self.tile = np.arange(F * Q).reshape(F, Q)
        self.pal = v.dith_pal.reshape(F, Q).astype(np.int64)
        self.hm = np.zeros((F, Q), np.uint8)
        self.vm = np.zeros((F, Q), np.uint8)

    def _remap(self, mi):
        m = np.asarray(mi)[self.tile]
        self.tile = np.where(m >= 0, m, self.tile)

    def unique(self, oracle, first, count):
        s = slice(first, first + count)
        pp, act, uc, mi = oracle.make_tiles_unique(self.palpix[s], self.active[s], self.uc[s])
        self.palpix[s], self.active[s], self.uc[s] = pp, act, uc
        full = np.full(self.palpix.shape[0], -1)
        full[s] = np.where(mi >= 0, mi + first, -1)
        self._remap(full)

    def pack(self, oracle):
        idx = oracle.reindex(self.active, self.uc)
        order = np.argsort(np.where(idx >= 0, idx, np.iinfo(np.int32).max), kind="stable")[: int((idx >= 0).sum())]
        self.palpix, self.thm, self.tvm = self.palpix[order], self.thm[order], self.tvm[order]
        self.dith, self.uc = self.dith[order], self.uc[order]
        self.active = np.ones(order.size, np.uint8)
        assert (idx[self.tile] >= 0).all()
        self.tile = idx[self.tile]

    def run(self, oracle, desired, quality, strength):
        v, Q = self.v, self.v.tiles_per_frame
        T0 = self.palpix.shape[0]
        for first in range(0, T0, Q * 25):
            self.unique(oracle, first, min(Q * 25, T0 - first))
        snap = {"unique": (self.active.copy(), self.tile.copy())}
        pp, act, uc, mi, _ = oracle.global_tiling(self.palpix, self.dith, v.palettes.shape[1], desired,
                                                  use_count=self.uc, active=self.active)
        self.palpix, self.active, self.uc = pp, act, uc
        self._remap(mi)
        self.unique(oracle, 0, self.palpix.shape[0])
        self.pack(oracle)
        snap["global"] = (self.palpix.copy(), self.uc.copy(), self.tile.copy())
        gds, gt_, ga = oracle.prepare_global_ds(self.palpix)
        for k in range(v.kf_start.size - 1):
            f0, f1 = int(v.kf_start[k]), int(v.kf_start[k + 1])
            corr, hi = oracle.palette_corr(v.centroids[k])
            used = oracle.mark_used(gds, gt_, ga, self.pal[f0:f1].ravel(), self.tile[f0:f1].ravel(), self.palpix,
                                    v.palettes.shape[1], quality, corr, hi)
            ds, ti, pi, at = oracle.build_ft_dataset(used, self.palpix, self.thm, self.tvm, v.palettes[k])
            t, p, h, vv, _ = oracle.frame_tiling(v.frame_rgb[f0:f1], ds, ti, pi, at)
            n = (f1 - f0, Q)
            self.tile[f0:f1], self.pal[f0:f1] = t.reshape(n), p.reshape(n)
            self.hm[f0:f1], self.vm[f0:f1] = h.reshape(n), vv.reshape(n)
        snap["ft"] = (self.tile.copy(), self.pal.copy(), self.hm.copy(), self.vm.copy())
        self.uc = np.bincount(self.tile.ravel(), minlength=self.palpix.shape[0]).astype(np.int32)
        self.active = (self.uc > 0).astype(np.uint8)
        self.pack(oracle)
        snap["reindex"] = (self.palpix.copy(), self.tile.copy())
        sm = [self.tile.copy(), self.pal.copy(), self.hm.copy(), self.vm.copy(), np.zeros(self.tile.shape, np.uint8)]
        for k in range(v.kf_start.size - 1):
            f0, f1 = int(v.kf_start[k]), int(v.kf_start[k + 1])
            out = oracle.smooth(*[a[f0:f1] for a in sm], self.palpix, v.palettes[k], strength)
            for a, b in zip(sm, out[:5]):
                a[f0:f1] = b
        snap["smooth"] = tuple(sm)
        return snap


@pytest.mark.gpu
@pytest.mark.parametrize("quality", [FT_MEDIUM, FT_FAST, FT_SLOW])
def test_run_all_chain_bit_exact(gpu, oracle, quality):
    from tiler_amd.encoder import Encoder
    v = synth.video(51 + quality, 320, 240, kf_frames=(3, 3), n_palettes=8)
    desired, strength = 700, 0.2
    o = _OracleChain(v).run(oracle, desired, quality, strength)

    e = Encoder(v)
    e.do_make_unique()
    assert np.array_equal(e.active, o["unique"][0]) and np.array_equal(e.tile, o["unique"][1])
    assert e.active.sum() < e.active.size  # frames repeat tiles: MakeUnique merged some
    e.do_global_tiling(desired)
    assert np.array_equal(e.palpix, o["global"][0])
    assert np.array_equal(e.use_count, o["global"][1])
    assert np.array_equal(e.tile, o["global"][2])
    assert e.palpix.shape[0] <= desired + v.palettes.shape[1]
    e.do_frame_tiling(quality)
    for a, b in zip((e.tile, e.pal, e.hm, e.vm), o["ft"]):
        assert np.array_equal(a, b)
    e.do_reindex()
    assert np.array_equal(e.palpix, o["reindex"][0]) and np.array_equal(e.tile, o["reindex"][1])
    sm = e.do_smooth(strength)
    for a, b in zip((sm["tile"], sm["pal"], sm["hm"], sm["vm"], sm["smoothed"]), o["smooth"]):
        assert np.array_equal(a, b)
    assert sm["smoothed"].sum() > 0
    # SaveStream: the .gtm carries exactly the SmoothedTileMap items
    from gtm_read import read_gtm
    g = read_gtm(oracle, e.save_stream(320, 240, 24.0))
    assert len(g.frames) == e.frames and np.array_equal(g.tiles, e.palpix)
    for f, (items, _, _) in enumerate(g.frames):
        live = ~sm["smoothed"][f].astype(bool)
        assert np.array_equal(items[:, 0] >= 0, live)
        t = sm["tile"][f]
        attrs = (sm["pal"][f] << 2) | ((sm["vm"][f] ^ e.tvm[t]) << 1) | (sm["hm"][f] ^ e.thm[t])
        assert np.array_equal(items[live, 0], t[live]) and np.array_equal(items[live, 1], attrs[live])


def _dist_worker(rank, world, port, out, quality, backend="gloo"):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(0)  # RCCL: the collective tensors live in this rank's HBM (dist.comm_device)
    dist.init_process_group(backend, rank=rank, world_size=world)
    import tiler_amd
    from tiler_amd import dist as td
    from tiler_amd._lib import check
    from tiler_amd.encoder import DistributedEncoder
    check(tiler_amd.load().tiler_init(0), "tiler_init")  # every rank on the one GPU of the test box
    v = synth.video(61, 320, 240, kf_frames=(3, 2, 3), n_palettes=8)
    e = DistributedEncoder(v, device=0)
    sm = e.run_all(700, quality, 0.2)
    data = e.save_stream(320, 240, 24.0)  # a collective: every rank calls it, rank 0 gets the bytes
    assert e.frames == e.frame_idx.size
    if world > 1:
        assert e.frame_idx.size < v.frames  # only this rank's keyframes are held
    # the reduced tileset from rank 0 (the north star's tileset exchange), through the backend's device
    tiles = td.broadcast_array(e.palpix if rank == 0 else None, e.palpix.shape, e.palpix.dtype)
    assert np.array_equal(tiles, e.palpix)
    np.savez(out + f".{rank}.npz", frame_idx=e.frame_idx, palpix=e.palpix, tile=e.tile, pal=e.pal, hm=e.hm, vm=e.vm,
             sm_tile=sm["tile"], sm_smoothed=sm["smoothed"], comm_device=str(td.comm_device()),
             backend=dist.get_backend(),
             gtm=np.frombuffer(data, np.uint8) if data is not None else np.zeros(0, np.uint8))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_run_all_chain_two_ranks_match_single_process(gpu, tmp_path):
    """the chain with palette bins and keyframes sharded over 2 ranks (gloo, both ranks on
    the test box's one GPU) ends in exactly the single-process state and .gtm bytes."""
    import socket
    import torch.multiprocessing as mp
    from tiler_amd.encoder import Encoder
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "r.npz")
    mp.spawn(_dist_worker, args=(2, port, out, FT_MEDIUM), nprocs=2, join=True)
    v = synth.video(61, 320, 240, kf_frames=(3, 2, 3), n_palettes=8)
    e = Encoder(v)
    sm = e.run_all(700, FT_MEDIUM, 0.2)
    data = e.save_stream(320, 240, 24.0)
    seen = np.zeros(v.frames, bool)
    for rank in range(2):
        got = np.load(out + f".{rank}.npz")
        fi = got["frame_idx"]
        seen[fi] = True
        assert np.array_equal(got["palpix"], e.palpix)  # the reduced tileset is replicated
        for k, a in (("tile", e.tile), ("pal", e.pal), ("hm", e.hm), ("vm", e.vm), ("sm_tile", sm["tile"]),
                     ("sm_smoothed", sm["smoothed"])):
            assert np.array_equal(got[k], a[fi]), (rank, k)
        if rank == 0:
            assert got["gtm"].tobytes() == data
        else:
            assert got["gtm"].size == 0
    assert seen.all()


@pytest.mark.gpu
def test_run_all_chain_nccl_world1_matches_single_process(gpu, tmp_path):
    """The product's RCCL branch executed: DistributedEncoder at world size 1 on the nccl
    backend -- the merge-map MAX and UseCount SUM all-reduces, gather_units' stream lengths and the tileset broadcast
    run as device tensors through RCCL (dist.comm_device = the rank's GPU) -- ends in exactly the single-process state
    and .gtm bytes."""
    import socket
    import torch.multiprocessing as mp
    from tiler_amd.encoder import Encoder
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "n.npz")
    mp.spawn(_dist_worker, args=(1, port, out, FT_MEDIUM, "nccl"), nprocs=1, join=True)
    v = synth.video(61, 320, 240, kf_frames=(3, 2, 3), n_palettes=8)
    e = Encoder(v)
    sm = e.run_all(700, FT_MEDIUM, 0.2)
    data = e.save_stream(320, 240, 24.0)
    got = np.load(out + ".0.npz")
    assert str(got["backend"]) == "nccl" and str(got["comm_device"]).startswith("cuda")
    assert np.array_equal(got["frame_idx"], np.arange(v.frames))
    assert np.array_equal(got["palpix"], e.palpix)
    for k, a in (("tile", e.tile), ("pal", e.pal), ("hm", e.hm), ("vm", e.vm), ("sm_tile", sm["tile"]),
                 ("sm_smoothed", sm["smoothed"])):
        assert np.array_equal(got[k], a), k
    assert got["gtm"].tobytes() == data


@pytest.mark.gpu
def test_load_dither_chain(gpu, oracle):
    """Load (keyframe split) and Dither (Thomas Knoll + mirrors) on the GPU in front of the chain: the Video
    equals the one composed from the CPU restatements, and the chain runs on it to a decodable .gtm."""
    from tiler_amd.encoder import Encoder, load_and_dither
    rng = np.random.default_rng(77)
    tm_w, tm_h = 20, 15
    frames, starts = synth.shot_frames(rng, 12, tm_w, tm_h, shot_len=(4, 6))
    pal_rng = lambda k: np.random.default_rng(1000 + k)  # noqa: E731
    pf = lambda k, fr: synth.palettes(pal_rng(k), 8)     # noqa: E731
    v = load_and_dither(frames, tm_w, tm_h, pf)
    okf, nkf = oracle.find_keyframes(oracle.interframe_corr_batch(frames, tm_w, tm_h), 12, tm_w * tm_h)
    opals = np.stack([pf(k, None) for k in range(nkf)])
    ov = synth.video_from_frames(frames, okf, opals, oracle.dither_tiles_tk)
    assert np.array_equal(v.kf_start, ov.kf_start) and set(starts.tolist()) <= set(v.kf_start[:-1].tolist())
    for a, b in ((v.palpix, ov.palpix), (v.thm, ov.thm), (v.tvm, ov.tvm), (v.dith_pal, ov.dith_pal)):
        assert np.array_equal(a, b)
    o = _OracleChain(ov).run(oracle, 500, FT_MEDIUM, 0.2)
    e = Encoder(v)
    sm = e.run_all(500, FT_MEDIUM, 0.2)
    for a, b in zip((sm["tile"], sm["pal"], sm["hm"], sm["vm"], sm["smoothed"]), o["smooth"]):
        assert np.array_equal(a, b)
    from gtm_read import read_gtm
    g = read_gtm(oracle, e.save_stream(tm_w * 8, tm_h * 8, 24.0))
    assert len(g.frames) == e.frames and np.array_equal(g.tiles, e.palpix)


@pytest.mark.gpu
def test_load_dither_generated_palettes_chain(gpu, oracle):
    """SURVEY.md 8(f)-3 complete: Load -> Dither with GPU-generated palettes (PrepareDitherTiles' k-means over LAB
    descriptors, QuantizePalette DLv3, FinishQuantizePalette, FinishDitherTiles) -> MakeUnique -> GlobalTiling ->
    FrameTiling (Medium: uses the generated PaletteCentroids) -> Reindex -> Smooth -> SaveStream, bit-exact against
    the same chain composed from the CPU restatements."""
    from tiler_amd.encoder import Encoder, load_and_dither
    rng = np.random.default_rng(79)
    tm_w, tm_h = 20, 15
    frames, _ = synth.shot_frames(rng, 10, tm_w, tm_h, shot_len=(4, 6))
    v = load_and_dither(frames, tm_w, tm_h, n_palettes=8)
    okf, nkf = oracle.find_keyframes(oracle.interframe_corr_batch(frames, tm_w, tm_h), 10, tm_w * tm_h)
    kf_start = np.r_[np.flatnonzero(np.r_[True, okf[1:] != okf[:-1]]), 10]
    opals, ocents, odith, _ = oracle.generate_palettes(frames, kf_start, 8)
    ov = synth.video_from_dither(frames, kf_start, opals, ocents, odith, oracle.dither_tiles_tk)
    assert np.array_equal(v.kf_start, ov.kf_start)
    for a, b in ((v.palettes, ov.palettes), (v.centroids, ov.centroids), (v.dith_pal, ov.dith_pal),
                 (v.palpix, ov.palpix), (v.thm, ov.thm), (v.tvm, ov.tvm)):
        assert np.array_equal(a, b)
    o = _OracleChain(ov).run(oracle, 500, FT_MEDIUM, 0.2)
    e = Encoder(v)
    sm = e.run_all(500, FT_MEDIUM, 0.2)
    for a, b in zip((sm["tile"], sm["pal"], sm["hm"], sm["vm"], sm["smoothed"]), o["smooth"]):
        assert np.array_equal(a, b)
    from gtm_read import read_gtm
    g = read_gtm(oracle, e.save_stream(tm_w * 8, tm_h * 8, 24.0))
    assert len(g.frames) == e.frames and np.array_equal(g.tiles, e.palpix)

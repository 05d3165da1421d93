"""The encoder steps around the hot path, end to end (btnRunAllClick main.pas:1232-1272, steps
MakeUnique -> GlobalTiling -> FrameTiling -> Reindex -> Smooth), as host state + libANN.so calls.

`Encoder` holds what TMainForm keeps in FTiles / FFrames / FKeyFrames for these steps, as flat arrays:
  tiles    palpix [T][64] u8, thm/tvm (TTile.HMirror/VMirror), active, use_count, dith_pal
  tilemaps tile/pal/hm/vm [F][Q] (TFrame.TileMap), sm_* the SmoothedTileMap copies
  keyframes kf_start [KF+1], palettes [KF][P][16], centroids [KF][P][192]
Each method is the reference procedure of the same name (file:line in its docstring); the heavy parts
(K-Modes, the k=8 preselection, candidate descriptors, the FrameTiling search, Smooth) run on the GPU
through the C ABI, the rest is the reference's host bookkeeping.  SURVEY.md 8(f)-1.
"""
from __future__ import annotations

import numpy as np

from . import frame_tiling as ft
from . import global_tiling as gt
from .gtm import save_stream
from .smooth import DEFAULT_STRENGTH, smooth_keyframe
from .synth import Video, video_from_frames


def load_and_dither(frames, tm_w: int, tm_h: int, palettes_fn=None, n_palettes: int = 8, gamma: int = -1,
                    use_wavelets: bool = True) -> Video:
    """The Load and Dither steps in front of the chain on the GPU (btnLoadClick main.pas:1099-1146, btnDitherClick
    main.pas:858-914): keyframes from the inter-frame correlations, then the keyframe palettes -- PrepareDitherTiles
    (LAB descriptors + k-means -> DitheringPalIndex, PaletteCentroids), QuantizePalette (DLv3), FinishQuantizePalette
    (tiler_amd.palette) -- and every tile dithered with its palette (FinishDitherTiles).  palettes_fn(k,
    frames_of_keyframe) -> [P][16], when given, replaces the palette generation (with the stand-in palette choice
    of synth.video_from_frames)."""
    from .dither import dither_tiles
    from .keyframes import detect_keyframes
    from .palette import generate_palettes
    from .synth import video_from_dither
    frames = np.ascontiguousarray(frames, np.int32).reshape(-1, tm_w * tm_h, 64)
    kf_of, kf_start, _ = detect_keyframes(frames, tm_w, tm_h)
    if palettes_fn is not None:
        pals = np.stack([np.asarray(palettes_fn(k, frames[kf_start[k]:kf_start[k + 1]]), np.int32)
                         for k in range(kf_start.size - 1)])
        return video_from_frames(frames, kf_of, pals, dither_tiles)
    pals, cents, dith, _ = generate_palettes(frames, kf_start, n_palettes, gamma=gamma, use_wavelets=use_wavelets)
    return video_from_dither(frames, kf_start, pals, cents, dith, dither_tiles)


class Encoder:
    def __init__(self, v: Video, palsize: int = 16):
        F, Q = v.frames, v.tiles_per_frame
        self.palsize = palsize
        self.frame_rgb = v.frame_rgb
        self.kf_start = np.asarray(v.kf_start, np.int64)
        self.palettes = np.asarray(v.palettes, np.int32)
        self.centroids = np.asarray(v.centroids, np.float64)
        self.n_palettes = self.palettes.shape[1]
        # FTiles after Dither (LoadFrame main.pas:3226-3236 + FinishDitherTiles 2497-2519)
        self.palpix = np.array(v.palpix, np.uint8, copy=True)
        self.thm = np.array(v.thm, np.uint8, copy=True)
        self.tvm = np.array(v.tvm, np.uint8, copy=True)
        self.dith_pal = np.array(v.dith_pal, np.int32, copy=True)
        self.active = np.ones(F * Q, np.uint8)
        self.use_count = np.ones(F * Q, np.int64)
        # TileMap: GlobalTileIndex = own tile, PalIdx = DitheringPalIndex, mirrors false
        self.tile = np.arange(F * Q, dtype=np.int64).reshape(F, Q)
        self.pal = self.dith_pal.reshape(F, Q).astype(np.int64)
        self.hm = np.zeros((F, Q), np.uint8)
        self.vm = np.zeros((F, Q), np.uint8)
        self.sm = None

    @property
    def frames(self) -> int:
        return self.tile.shape[0]

    @property
    def tiles_per_frame(self) -> int:
        return self.tile.shape[1]

    # --- tile-list bookkeeping --------------------------------------------------------------------
    def finish_merge_tiles(self, merge_index):
        """FinishMergeTiles main.pas:3722-3734: TileMap items of merged tiles point at the survivor."""
        m = np.asarray(merge_index, np.int64)[self.tile]
        self.tile = np.where(m >= 0, m, self.tile)

    def make_tiles_unique(self, first: int = 0, count: int | None = None):
        """MakeTilesUnique main.pas:2555-2612 over tiles [first, first+count): identical PalPixels merge
        into the lowest index (TFPList.Sort is unstable, the canonical order is stable)."""
        count = self.palpix.shape[0] - first if count is None else count
        s = slice(first, first + count)
        pp, act, uc, mi = gt.make_tiles_unique(self.palpix[s], self.active[s], self.use_count[s])
        self.palpix[s], self.active[s], self.use_count[s] = pp, act, uc
        full = np.full(self.palpix.shape[0], -1, np.int64)
        full[s] = np.where(mi >= 0, mi + first, -1)
        self.finish_merge_tiles(full)

    def reindex_tiles(self):
        """ReindexTiles main.pas:4483-4527: drop inactive tiles, order by (UseCount desc, old index asc),
        remap every TileMap."""
        idx_map = gt.reindex_tiles(self.active, self.use_count)
        keep = np.nonzero(idx_map >= 0)[0]
        order = np.empty(keep.size, np.int64)
        order[idx_map[keep]] = keep
        self.palpix = np.ascontiguousarray(self.palpix[order])
        self.thm, self.tvm = self.thm[order], self.tvm[order]
        self.dith_pal, self.use_count = self.dith_pal[order], self.use_count[order]
        self.active = np.ones(order.size, np.uint8)
        self.tile = idx_map[self.tile]
        if self.sm is not None:
            self.sm["tile"] = idx_map[self.sm["tile"]]

    # --- steps ------------------------------------------------------------------------------------
    def do_make_unique(self):
        """btnDoMakeUniqueClick main.pas:916-938: MakeTilesUnique per chunk of FTileMapSize * 25 tiles."""
        chunk = self.tiles_per_frame * 25
        for first in range(0, self.palpix.shape[0], chunk):
            self.make_tiles_unique(first, min(chunk, self.palpix.shape[0] - first))

    def do_global_tiling(self, desired: int, restart: int = gt.CRANDOM_KMODES_COUNT):
        """DoGlobalTiling main.pas:4256-4370: K-Modes merge per palette bin (GPU, all bins batched),
        FinishMergeTiles, MakeTilesUnique over all tiles, ReindexTiles."""
        pp, act, uc, mi, kpb = gt.do_global_tiling(self.palpix, self.dith_pal, self.n_palettes, desired,
                                                   self.palsize, restart, self.active, self.use_count)
        self.palpix, self.active, self.use_count = pp, act, uc
        self.finish_merge_tiles(mi)
        self.make_tiles_unique()
        self.reindex_tiles()
        return kpb

    def do_frame_tiling(self, quality: int = ft.FT_MEDIUM, use_wavelets: bool = True, gamma: int = -1):
        """btnDoFrameTilingClick main.pas:945-977: PrepareGlobalFT, then per keyframe PrepareFrameTiling
        (over the keyframe's current TileMap items), DoFrameTiling of all its frames, FinishFrameTiling."""
        gds = ft.prepare_global_ft(self.palpix, self.active)
        errs = np.zeros(self.tile.shape, np.float32)
        try:
            for k in range(self.kf_start.size - 1):
                f0, f1 = int(self.kf_start[k]), int(self.kf_start[k + 1])
                kt = ft.prepare_frame_tiling(self.palpix, self.thm, self.tvm, self.palettes[k], gds,
                                             self.pal[f0:f1].ravel(), self.tile[f0:f1].ravel(), quality,
                                             self.centroids[k], use_wavelets, gamma)
                try:
                    t, p, h, v, e = kt.do_frame_tiling(self.frame_rgb[f0:f1])
                finally:
                    kt.finish_frame_tiling()
                n = (f1 - f0, self.tiles_per_frame)
                self.tile[f0:f1], self.pal[f0:f1] = t.reshape(n), p.reshape(n)
                self.hm[f0:f1], self.vm[f0:f1], errs[f0:f1] = h.reshape(n), v.reshape(n), e.reshape(n)
        finally:
            gds.kdt.close()
        return errs

    def do_reindex(self):
        """btnReindexClick main.pas:1199-1230: UseCount / Active from the TileMaps, then ReindexTiles."""
        T = self.palpix.shape[0]
        self.use_count = np.bincount(self.tile.ravel(), minlength=T).astype(np.int64)
        self.active = (self.use_count > 0).astype(np.uint8)
        self.reindex_tiles()

    def do_smooth(self, strength: float = DEFAULT_STRENGTH):
        """btnSmoothClick main.pas:1338-1370: SmoothedTileMap := TileMap, then DoTemporalSmoothing along
        every position (frames of one keyframe only, main.pas:4081-4082) -> one GPU call per keyframe."""
        sm = {"tile": self.tile.copy(), "pal": self.pal.copy(), "hm": self.hm.copy(), "vm": self.vm.copy(),
              "smoothed": np.zeros(self.tile.shape, np.uint8)}
        for k in range(self.kf_start.size - 1):
            f0, f1 = int(self.kf_start[k]), int(self.kf_start[k + 1])
            t, p, h, v, s, _ = smooth_keyframe(sm["tile"][f0:f1], sm["pal"][f0:f1], sm["hm"][f0:f1],
                                               sm["vm"][f0:f1], sm["smoothed"][f0:f1], self.palpix,
                                               self.palettes[k], strength)
            sm["tile"][f0:f1], sm["pal"][f0:f1], sm["hm"][f0:f1], sm["vm"][f0:f1] = t, p, h, v
            sm["smoothed"][f0:f1] = s
        self.sm = sm
        return sm

    def save_stream(self, width: int, height: int, fps: float = 24.0) -> bytes:
        """btnSaveClick -> SaveStream main.pas:4529-4763 (the .gtm bytes; needs do_smooth first)."""
        sm = self.sm
        return save_stream(self.palpix, self.thm, self.tvm, self.kf_start, self.palettes, sm["tile"], sm["pal"],
                           sm["hm"], sm["vm"], sm["smoothed"], width, height, fps, self.palsize)

    def run_all(self, desired: int, quality: int = ft.FT_MEDIUM, strength: float = DEFAULT_STRENGTH):
        """btnRunAllClick main.pas:1232-1272 from MakeUnique to Smooth."""
        self.do_make_unique()
        self.do_global_tiling(desired)
        self.do_frame_tiling(quality)
        self.do_reindex()
        return self.do_smooth(strength)


class DistributedEncoder(Encoder):
    """The same chain with one process per GPU (tiler_amd.dist).  Call inside an initialised
    torch.distributed process group (backend "nccl" = RCCL over xGMI; "gloo" for CPU-side tests).

    Device: each rank binds its own GPU -- libANN.so through tiler_init(device) and torch through
    torch.cuda.set_device(device) -- with device = LOCAL_RANK (torchrun's one process per GPU) unless given.
    Work: palette bins (K-Modes) and keyframes (FrameTiling, then Smooth, same plan) are assigned longest-first
    across the ranks; a rank computes only its own units.  Exchanges (fixed-layout tensors, tiler_amd.dist):
    the K-Modes merge map (all-reduce MAX) so every rank holds the reduced tileset, the UseCount histogram
    (all-reduce SUM) for ReindexTiles, and the tilemaps onto rank `save_rank` only (reduce SUM) for SaveStream.
    Between steps a rank's tilemaps are current for its own keyframes only; after run_all (or gather()) rank
    `save_rank` holds the whole single-process state."""

    def __init__(self, v: Video, palsize: int = 16, device: int | None = None, save_rank: int = 0):
        import os

        import torch
        import torch.distributed as dist

        from ._lib import check, load
        from . import dist as tdist
        super().__init__(v, palsize)
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.device = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
        check(load().tiler_init(self.device), "tiler_init")
        if torch.cuda.is_available():
            torch.cuda.set_device(self.device)
        self.save_rank = save_rank
        nkf = self.kf_start.size - 1
        kf_frames = [int(self.kf_start[k + 1] - self.kf_start[k]) for k in range(nkf)]
        self.my_kf = tdist.plan_keyframes(kf_frames, self.tiles_per_frame, self.world)[self.rank]
        self.my_frames = np.zeros(self.frames, bool)
        for k in self.my_kf:
            self.my_frames[int(self.kf_start[k]):int(self.kf_start[k + 1])] = True

    def do_global_tiling(self, desired: int, restart: int = gt.CRANDOM_KMODES_COUNT):
        from . import dist as tdist
        plan = gt.plan_global_tiling(self.palpix, self.dith_pal, self.n_palettes, desired, self.palsize, restart,
                                     self.active)
        run = plan.run
        costs = [plan.bins[p].size * max(1, int(plan.k_per_bin[p])) for p in run]
        mine = [run[u] for u in tdist.lpt_assign(costs, self.world)[self.rank]]
        local = gt.kmodes_bins(plan, mine, self.palsize)  # this rank's bins in one GPU batch
        merge_to = tdist.allreduce(gt.kmodes_merge_map(plan, local, self.palpix.shape[0]), "max")
        pp, act, uc, mi = gt.apply_merge_map(merge_to, self.palpix, self.active, self.use_count)
        self.palpix, self.active, self.use_count = pp, act, uc
        self.finish_merge_tiles(mi)
        self.make_tiles_unique()
        self.reindex_tiles()
        return plan.k_per_bin

    def do_frame_tiling(self, quality: int = ft.FT_MEDIUM, use_wavelets: bool = True, gamma: int = -1):
        """This rank's keyframes only (their TileMaps become current; the others' stay as they were)."""
        gds = ft.prepare_global_ft(self.palpix, self.active)
        errs = np.zeros(self.tile.shape, np.float32)
        Q = self.tiles_per_frame
        try:
            for k in self.my_kf:
                f0, f1 = int(self.kf_start[k]), int(self.kf_start[k + 1])
                kt = ft.prepare_frame_tiling(self.palpix, self.thm, self.tvm, self.palettes[k], gds,
                                             self.pal[f0:f1].ravel(), self.tile[f0:f1].ravel(), quality,
                                             self.centroids[k], use_wavelets, gamma)
                try:
                    t, p, h, v, e = kt.do_frame_tiling(self.frame_rgb[f0:f1])
                finally:
                    kt.finish_frame_tiling()
                n = (f1 - f0, Q)
                self.tile[f0:f1], self.pal[f0:f1] = t.reshape(n), p.reshape(n)
                self.hm[f0:f1], self.vm[f0:f1], errs[f0:f1] = h.reshape(n), v.reshape(n), e.reshape(n)
        finally:
            gds.kdt.close()
        return errs

    def do_reindex(self):
        """btnReindexClick main.pas:1199-1230 with the UseCount histogram all-reduced over the ranks' keyframes."""
        from . import dist as tdist
        T = self.palpix.shape[0]
        local = np.bincount(self.tile[self.my_frames].ravel(), minlength=T).astype(np.int64)
        self.use_count = tdist.allreduce(local, "sum")
        self.active = (self.use_count > 0).astype(np.uint8)
        self.tile = np.where(self.my_frames[:, None], self.tile, 0)  # other ranks' frames: not current here
        self.reindex_tiles()

    def do_smooth(self, strength: float = DEFAULT_STRENGTH):
        sm = {"tile": self.tile.copy(), "pal": self.pal.copy(), "hm": self.hm.copy(), "vm": self.vm.copy(),
              "smoothed": np.zeros(self.tile.shape, np.uint8)}
        for k in self.my_kf:
            f0, f1 = int(self.kf_start[k]), int(self.kf_start[k + 1])
            t, p, h, v, s, _ = smooth_keyframe(sm["tile"][f0:f1], sm["pal"][f0:f1], sm["hm"][f0:f1],
                                               sm["vm"][f0:f1], sm["smoothed"][f0:f1], self.palpix,
                                               self.palettes[k], strength)
            sm["tile"][f0:f1], sm["pal"][f0:f1], sm["hm"][f0:f1], sm["vm"][f0:f1] = t, p, h, v
            sm["smoothed"][f0:f1] = s
        self.sm = sm
        return sm

    def gather(self):
        """Every rank's keyframes' TileMaps and SmoothedTileMaps onto rank save_rank (one reduce of int32
        [F][Q][4]: tile, pal | hm << 16 | vm << 17, and the same for the smoothed items | smoothed << 18)."""
        from . import dist as tdist
        if self.n_palettes > 1 << 16:
            raise ValueError("palette index does not fit the packed tilemap layout")
        own = self.my_frames[:, None]
        sm = self.sm
        pk = np.zeros(self.tile.shape + (4,), np.int32)
        pk[..., 0] = np.where(own, self.tile, 0)
        pk[..., 1] = np.where(own, self.pal | (self.hm.astype(np.int64) << 16) | (self.vm.astype(np.int64) << 17), 0)
        if sm is not None:
            pk[..., 2] = np.where(own, sm["tile"], 0)
            pk[..., 3] = np.where(own, sm["pal"] | (sm["hm"].astype(np.int64) << 16) |
                                  (sm["vm"].astype(np.int64) << 17) | (sm["smoothed"].astype(np.int64) << 18), 0)
        full = tdist.reduce_to(pk, self.save_rank)
        if full is None:
            return None
        self.tile = full[..., 0].astype(np.int64)
        self.pal = (full[..., 1] & 0xFFFF).astype(np.int64)
        self.hm = ((full[..., 1] >> 16) & 1).astype(np.uint8)
        self.vm = ((full[..., 1] >> 17) & 1).astype(np.uint8)
        self.my_frames[:] = True
        if sm is not None:
            self.sm = {"tile": full[..., 2].astype(np.int64), "pal": (full[..., 3] & 0xFFFF).astype(np.int64),
                       "hm": ((full[..., 3] >> 16) & 1).astype(np.uint8),
                       "vm": ((full[..., 3] >> 17) & 1).astype(np.uint8),
                       "smoothed": ((full[..., 3] >> 18) & 1).astype(np.uint8)}
        return self.sm

    def run_all(self, desired: int, quality: int = ft.FT_MEDIUM, strength: float = DEFAULT_STRENGTH):
        """btnRunAllClick from MakeUnique to Smooth, then the tilemaps onto save_rank (None on the other ranks)."""
        super().run_all(desired, quality, strength)
        return self.gather()

    def save_stream(self, width: int, height: int, fps: float = 24.0) -> bytes:
        if self.rank != self.save_rank:
            raise RuntimeError(f"SaveStream runs on rank {self.save_rank}, which holds the gathered tilemaps")
        return super().save_stream(width, height, fps)

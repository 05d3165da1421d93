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
from . import gtm
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
    """frames: the global frame indices this encoder holds the frames and tilemaps of (sorted, whole keyframes;
    None = all).  The tileset (palpix, flags, Active, UseCount) is always the whole clip's.  Tilemap arrays are
    [len(frames)][Q]: row r is frame frames[r]."""

    def __init__(self, v: Video, palsize: int = 16, frames=None):
        F, Q = v.frames, v.tiles_per_frame
        self.palsize = palsize
        self.n_frames = F
        self.kf_start = np.asarray(v.kf_start, np.int64)
        own = np.arange(F) if frames is None else np.asarray(frames, np.int64)
        self.frame_idx = own
        # only the held frames are read (a memory-mapped Video pages in just these)
        self.frame_rgb = v.frame_rgb if frames is None else np.ascontiguousarray(v.frame_rgb[own])
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
        self.tile = (own[:, None] * Q + np.arange(Q, dtype=np.int64)[None, :])
        self.pal = self.dith_pal.reshape(F, Q)[own].astype(np.int64)
        self.hm = np.zeros((own.size, Q), np.uint8)
        self.vm = np.zeros((own.size, Q), np.uint8)
        self.sm = None
        # the keyframes held (every frame of each), and their first tilemap row
        self.kfs = [k for k in range(self.kf_start.size - 1)
                    if np.isin(np.arange(self.kf_start[k], self.kf_start[k + 1]), own).all()]
        self._row0 = {k: int(np.searchsorted(own, self.kf_start[k])) for k in self.kfs}
        if sum(int(self.kf_start[k + 1] - self.kf_start[k]) for k in self.kfs) != own.size:
            raise ValueError("an encoder holds whole keyframes only")

    @property
    def frames(self) -> int:
        return self.tile.shape[0]

    @property
    def tiles_per_frame(self) -> int:
        return self.tile.shape[1]

    def rows(self, k: int) -> slice:
        """Tilemap rows of keyframe k."""
        r0 = self._row0[k]
        return slice(r0, r0 + int(self.kf_start[k + 1] - self.kf_start[k]))

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
        Q = self.tiles_per_frame
        try:
            for k in self.kfs:
                r = self.rows(k)
                kt = ft.prepare_frame_tiling(self.palpix, self.thm, self.tvm, self.palettes[k], gds,
                                             self.pal[r].ravel(), self.tile[r].ravel(), quality,
                                             self.centroids[k], use_wavelets, gamma)
                try:
                    t, p, h, v, e = kt.do_frame_tiling(self.frame_rgb[r])
                finally:
                    kt.finish_frame_tiling()
                n = (r.stop - r.start, Q)
                self.tile[r], self.pal[r] = t.reshape(n), p.reshape(n)
                self.hm[r], self.vm[r], errs[r] = h.reshape(n), v.reshape(n), e.reshape(n)
        finally:
            gds.kdt.close()
        return errs

    def _use_count(self, T: int) -> np.ndarray:
        return np.bincount(self.tile.ravel(), minlength=T).astype(np.int64)

    def do_reindex(self):
        """btnReindexClick main.pas:1199-1230: UseCount / Active from the TileMaps, then ReindexTiles."""
        self.use_count = self._use_count(self.palpix.shape[0])
        self.active = (self.use_count > 0).astype(np.uint8)
        self.reindex_tiles()

    def do_smooth(self, strength: float = DEFAULT_STRENGTH):
        """btnSmoothClick main.pas:1338-1370: SmoothedTileMap := TileMap, then DoTemporalSmoothing along
        every position (frames of one keyframe only, main.pas:4081-4082) -> one GPU call per keyframe."""
        sm = {"tile": self.tile.copy(), "pal": self.pal.copy(), "hm": self.hm.copy(), "vm": self.vm.copy(),
              "smoothed": np.zeros(self.tile.shape, np.uint8)}
        for k in self.kfs:
            r = self.rows(k)
            t, p, h, v, s, _ = smooth_keyframe(sm["tile"][r], sm["pal"][r], sm["hm"][r], sm["vm"][r],
                                               sm["smoothed"][r], self.palpix, self.palettes[k], strength)
            sm["tile"][r], sm["pal"][r], sm["hm"][r], sm["vm"][r] = t, p, h, v
            sm["smoothed"][r] = s
        self.sm = sm
        return sm

    def _keyframe_streams(self, width: int, height: int, fps: float) -> dict:
        """LZCompress'd command stream of every held keyframe (SaveStream main.pas:4724-4734), compressed
        concurrently."""
        sm = self.sm
        if sm is None:
            raise RuntimeError("SaveStream needs the SmoothedTileMaps: run do_smooth first")
        raws = []
        for k in self.kfs:
            r = self.rows(k)
            raws.append(gtm.keyframe_raw(k, self.palpix, self.thm, self.tvm, self.palettes[k], sm["tile"][r],
                                         sm["pal"][r], sm["hm"][r], sm["vm"][r], sm["smoothed"][r], width=width,
                                         height=height, fps=fps, palsize=self.palsize))
        return dict(zip(self.kfs, gtm.compress_streams(raws)))

    def save_stream(self, width: int, height: int, fps: float = 24.0) -> bytes:
        """btnSaveClick -> SaveStream main.pas:4529-4763 (the .gtm bytes; needs do_smooth first)."""
        comps = self._keyframe_streams(width, height, fps)
        return gtm.assemble_stream([comps[k] for k in range(self.kf_start.size - 1)], self.kf_start, width, height,
                                   fps)

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
    across the ranks; a rank computes only its own units.  Memory: a rank holds the tileset (replicated, the north
    star's all-gathered tileset) and ONLY its own keyframes' frames and tilemaps ([own frames][Q]; `frame_idx`
    maps rows to frames).  Exchanges (fixed-layout tensors, tiler_amd.dist): the K-Modes merge map (all-reduce
    MAX) so every rank holds the reduced tileset, the UseCount histogram (all-reduce SUM) for ReindexTiles, and for
    SaveStream each rank's compressed keyframe streams onto rank `save_rank` (gather_units).  save_stream is a
    collective: every rank calls it, save_rank gets the .gtm bytes, the others None."""

    def __init__(self, v: Video, palsize: int = 16, device: int | None = None, save_rank: int = 0):
        import os

        import torch
        import torch.distributed as dist

        from ._lib import check, load
        from . import dist as tdist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        kf_start = np.asarray(v.kf_start, np.int64)
        nkf = kf_start.size - 1
        kf_frames = [int(kf_start[k + 1] - kf_start[k]) for k in range(nkf)]
        self.plan = tdist.plan_keyframes(kf_frames, v.tiles_per_frame, self.world)
        self.owner_of = [0] * nkf
        for r, units in enumerate(self.plan):
            for k in units:
                self.owner_of[k] = r
        mine = sorted(self.plan[self.rank])
        own = np.concatenate([np.arange(kf_start[k], kf_start[k + 1]) for k in mine]) if mine \
            else np.zeros(0, np.int64)
        super().__init__(v, palsize, frames=own)
        self.device = int(os.environ.get("LOCAL_RANK", "0")) if device is None else int(device)
        if self.device >= 0:  # device = -1: no GPU binding (host-side steps only, e.g. SaveStream in CPU tests)
            check(load().tiler_init(self.device), "tiler_init")
            if torch.cuda.is_available():
                torch.cuda.set_device(self.device)
        self.save_rank = save_rank

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

    def _use_count(self, T: int) -> np.ndarray:
        """btnReindexClick main.pas:1208-1221: the UseCount histogram over every rank's keyframes."""
        from . import dist as tdist
        return tdist.allreduce(super()._use_count(T), "sum")

    def save_stream(self, width: int, height: int, fps: float = 24.0) -> bytes | None:
        """SaveStream as a collective: every rank writes and compresses its own keyframes' streams, rank
        save_rank receives the others' and assembles the file (None on the other ranks)."""
        from . import dist as tdist
        comps = tdist.gather_units(self._keyframe_streams(width, height, fps), self.owner_of, self.save_rank)
        if comps is None:
            return None
        return gtm.assemble_stream(comps, self.kf_start, width, height, fps)

"""Seeded synthetic inputs for the tile-search hot path.

There is no video (ffmpeg.exe / Load step are out of scope), so frames, palettes and the global
tileset are generated with numpy's PCG64 from a recorded seed:
  - frame tiles: 50 % smooth gradients, 30 % textured (uniform +-32 around a per-tile mean), 20 % flat;
    frames of one keyframe evolve from the first (a share of tiles re-drawn per frame) so Smooth has work;
  - palettes: P x 16 uniform RGB (0x00BBGGRR, main.pas:566-569);
  - tileset: T random 4-bit index tiles, 20 % made H- and/or V-symmetric (exact mirror ties), then
    canonicalised like PrepareTileMirrors (main.pas:4049-4069); one palette per tile (P_eff = 1).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

TILE = 8


def rgb_pack(r, g, b):
    return (np.asarray(b, np.int32) << 16) | (np.asarray(g, np.int32) << 8) | np.asarray(r, np.int32)


def frame_tiles(rng: np.random.Generator, n: int) -> np.ndarray:
    """n RGB tiles [n, 64] int32 (0x00BBGGRR)."""
    kind = rng.random(n)
    out = np.empty((n, 64, 3), np.float64)
    yy, xx = np.mgrid[0:8, 0:8]
    yy = yy.reshape(64) / 7.0
    xx = xx.reshape(64) / 7.0
    grad = kind < 0.5
    tex = (kind >= 0.5) & (kind < 0.8)
    flat = kind >= 0.8
    ng = int(grad.sum())
    c0 = rng.integers(0, 256, (ng, 1, 3)).astype(np.float64)
    c1 = rng.integers(0, 256, (ng, 1, 3)).astype(np.float64)
    ang = rng.random((ng, 1, 1)) * 2 * np.pi
    t = (np.cos(ang) * xx[None, :, None] + np.sin(ang) * yy[None, :, None])
    t = (t - t.min(axis=1, keepdims=True)) / np.maximum(np.ptp(t, axis=1, keepdims=True), 1e-9)
    out[grad] = c0 + (c1 - c0) * t
    nt = int(tex.sum())
    mean = rng.integers(32, 224, (nt, 1, 3)).astype(np.float64)
    out[tex] = mean + rng.integers(-32, 33, (nt, 64, 3))
    nf = int(flat.sum())
    out[flat] = rng.integers(0, 256, (nf, 1, 3)).astype(np.float64)
    px = np.clip(np.rint(out), 0, 255).astype(np.int32)
    return rgb_pack(px[..., 0], px[..., 1], px[..., 2])


def keyframe_frames(rng: np.random.Generator, frames: int, tiles_per_frame: int, change: float = 0.3) -> np.ndarray:
    """[frames, Q, 64] int32; each frame re-draws `change` of the previous frame's tiles."""
    out = np.empty((frames, tiles_per_frame, 64), np.int32)
    out[0] = frame_tiles(rng, tiles_per_frame)
    for f in range(1, frames):
        out[f] = out[f - 1]
        sel = np.nonzero(rng.random(tiles_per_frame) < change)[0]
        if sel.size:
            out[f, sel] = frame_tiles(rng, sel.size)
    return out


def screen_to_tiles(img: np.ndarray) -> np.ndarray:
    """Screen [H][W][3] u8 (r, g, b) -> frame tiles [(H/8)*(W/8)][64] int32 0x00BBGGRR (LoadFrame main.pas:3245-3256)."""
    H, W, _ = img.shape
    t = img.reshape(H // 8, 8, W // 8, 8, 3).transpose(0, 2, 1, 3, 4).reshape(-1, 64, 3).astype(np.int32)
    return rgb_pack(t[..., 0], t[..., 1], t[..., 2])


def shot_frames(rng: np.random.Generator, frames: int, tm_w: int, tm_h: int, shot_len=(6, 40), noise: int = 6):
    """Synthetic clip with shot transitions for the Load step's keyframe detection: each shot is a smooth
    random picture that pans one pixel per frame under per-frame noise; a new shot starts after a random
    length.  Returns (frames [F][Q][64] int32, first frame of every shot)."""
    H, W = tm_h * 8, tm_w * 8
    out = np.empty((frames, tm_w * tm_h, 64), np.int32)
    starts = []
    f = 0
    while f < frames:
        starts.append(f)
        n = int(rng.integers(shot_len[0], shot_len[1] + 1))
        lo = rng.integers(0, 256, ((H + n) // 16 + 2, (W + 2 * n) // 16 + 2, 3)).astype(np.float32)
        base = np.repeat(np.repeat(lo, 16, 0), 16, 1)
        for k in range(min(n, frames - f)):
            img = base[k:k + H, 2 * k:2 * k + W]
            img = img + rng.integers(-noise, noise + 1, img.shape)
            out[f] = screen_to_tiles(np.clip(img, 0, 255).astype(np.uint8))
            f += 1
    return out, np.asarray(starts, np.int64)


def palettes(rng: np.random.Generator, count: int, size: int = 16) -> np.ndarray:
    c = rng.integers(0, 256, (count, size, 3))
    return rgb_pack(c[..., 0], c[..., 1], c[..., 2])


def hflip(t: np.ndarray) -> np.ndarray:
    return t.reshape(-1, 8, 8)[:, :, ::-1].reshape(t.shape)


def vflip(t: np.ndarray) -> np.ndarray:
    return t.reshape(-1, 8, 8)[:, ::-1, :].reshape(t.shape)


def prepare_tile_mirrors(pal_tiles: np.ndarray):
    """PrepareTileMirrors main.pas:4049-4069: pick the quadrant (v-outer, h-inner, first max) with the
    largest palette-index sum, flip it to the top-left; returns (tiles, HMirror, VMirror)."""
    t = pal_tiles.reshape(-1, 8, 8).astype(np.int64)
    sums = np.stack([t[:, 0:4, 0:4].sum((1, 2)), t[:, 0:4, 4:8].sum((1, 2)),
                     t[:, 4:8, 0:4].sum((1, 2)), t[:, 4:8, 4:8].sum((1, 2))], 1)  # order (vf,hf)=FF,FT,TF,TT
    best = np.argmax(sums, axis=1)  # first max == strict '>' scan in the reference
    hm = (best & 1).astype(np.uint8)
    vm = (best >> 1).astype(np.uint8)
    out = pal_tiles.copy()
    out[hm == 1] = hflip(out[hm == 1])
    out[vm == 1] = vflip(out[vm == 1])
    return out, hm, vm


def tileset(rng: np.random.Generator, count: int, palsize: int = 16, sym_share: float = 0.2):
    """[count, 64] uint8 palette-index tiles (canonical orientation) + HMirror/VMirror flags."""
    t = rng.integers(0, palsize, (count, 64)).astype(np.uint8).reshape(-1, 8, 8)
    kind = rng.random(count)
    hs = kind < sym_share * 0.4
    vs = (kind >= sym_share * 0.4) & (kind < sym_share * 0.8)
    hv = (kind >= sym_share * 0.8) & (kind < sym_share)
    t[hs, :, 4:] = t[hs, :, 3::-1]
    t[vs, 4:, :] = t[vs, 3::-1, :]
    t[hv, :, 4:] = t[hv, :, 3::-1]
    t[hv, 4:, :] = t[hv, 3::-1, :]
    tiles = t.reshape(count, 64)
    return prepare_tile_mirrors(tiles)


@dataclass
class FTDataset:
    """The keyframe search dataset of PrepareFrameTiling.DoPsyV (main.pas:3883-3919) as index arrays:
    candidate r = descriptor of tile_of[r] in palette pal_of[r] with attrs (H=1, V=2); psyv_flags[r] is
    the mirror actually applied (attrs xor the tile's canonical flags, main.pas:3912)."""
    tile_of: np.ndarray
    pal_of: np.ndarray
    attrs: np.ndarray
    psyv_flags: np.ndarray


def ft_dataset_from_used(used: np.ndarray, thm: np.ndarray, tvm: np.ndarray) -> FTDataset:
    """Emission order of DoPsyV: palette asc, tile asc, vmir F/T, hmir F/T (used[p, i, vm<<1|hm])."""
    P, T, _ = used.shape
    p, i, a = np.nonzero(used)  # row-major: p, then i, then a = (vm<<1)|hm ascending == vmir outer, hmir inner
    hm = (a & 1).astype(np.uint8)
    vm = ((a >> 1) & 1).astype(np.uint8)
    fl = (((hm ^ thm[i]) * 16) | ((vm ^ tvm[i]) * 32)).astype(np.uint8)
    return FTDataset(i.astype(np.int32), p.astype(np.int32), (hm | (vm << 1)).astype(np.uint8), fl)


def used_one_palette(tile_pal: np.ndarray, P: int) -> np.ndarray:
    """P_eff = 1 benchmark shape: every tile's 4 orientations used in its own palette only."""
    T = tile_pal.shape[0]
    used = np.zeros((P, T, 4), np.uint8)
    used[tile_pal, np.arange(T), :] = 1
    return used


@dataclass
class Workload:
    seed: int
    width: int
    height: int
    frames: int
    tileset_size: int
    palettes: np.ndarray
    tiles: np.ndarray
    thm: np.ndarray
    tvm: np.ndarray
    tile_pal: np.ndarray
    frame_rgb: np.ndarray  # [frames, Q, 64]
    ds: FTDataset

    @property
    def tiles_per_frame(self) -> int:
        return (self.width // TILE) * (self.height // TILE)


def make_workload(seed: int, width: int, height: int, frames: int, tileset_size: int, n_palettes: int = 128,
                  palsize: int = 16) -> Workload:
    rng = np.random.default_rng(seed)
    pals = palettes(rng, n_palettes, palsize)
    tiles, thm, tvm = tileset(rng, tileset_size, palsize)
    tile_pal = rng.integers(0, n_palettes, tileset_size).astype(np.int32)
    q = (width // TILE) * (height // TILE)
    fr = keyframe_frames(rng, frames, q)
    ds = ft_dataset_from_used(used_one_palette(tile_pal, n_palettes), thm, tvm)
    return Workload(seed, width, height, frames, tileset_size, pals, tiles, thm, tvm, tile_pal, fr, ds)


@dataclass
class Video:
    """Stand-in for the Load + Dither steps (out of scope): what btnRunAllClick hands
    to MakeUnique / GlobalTiling / FrameTiling.  Keyframe k owns frames kf_start[k]..kf_start[k+1]-1 and
    its palettes `palettes[k]` [P][16] + 192-d `centroids[k]`.  Every frame tile is one global tile
    (LoadFrame main.pas:3226-3236: tile f*Q+q), palettised by nearest colour in the keyframe palette with
    the lowest total error (NOT the reference's ditherer) and canonicalised like PrepareTileMirrors."""
    frame_rgb: np.ndarray      # [F][Q][64] int32
    kf_start: np.ndarray       # [KF+1]
    palettes: np.ndarray       # [KF][P][16] int32
    centroids: np.ndarray      # [KF][P][192] float64
    palpix: np.ndarray         # [F*Q][64] u8 (canonical orientation)
    thm: np.ndarray            # [F*Q] u8
    tvm: np.ndarray            # [F*Q] u8
    dith_pal: np.ndarray       # [F*Q] int32 (DitheringPalIndex)

    @property
    def frames(self) -> int:
        return self.frame_rgb.shape[0]

    @property
    def tiles_per_frame(self) -> int:
        return self.frame_rgb.shape[1]


def palette_centroids(pals: np.ndarray) -> np.ndarray:
    """Deterministic 192-d palette centroids (the reference takes yakmo's, main.pas:2477-2479): the 16
    colours sorted by luma, RGB/255, repeated 4x.  Close palettes get close centroids."""
    pals = np.asarray(pals, np.int64).reshape(-1, 16)
    rgb = np.stack([pals & 255, (pals >> 8) & 255, (pals >> 16) & 255], -1).astype(np.float64) / 255.0
    luma = rgb @ np.array([0.2126, 0.7152, 0.0722])
    order = np.argsort(luma, axis=1, kind="stable")
    srt = np.take_along_axis(rgb, order[..., None], 1).reshape(pals.shape[0], 48)
    return np.tile(srt, (1, 4))


def video(seed: int, width: int, height: int, kf_frames=(3, 3), n_palettes: int = 8, change: float = 0.3) -> Video:
    rng = np.random.default_rng(seed)
    q = (width // TILE) * (height // TILE)
    rgb, pals, starts = [], [], [0]
    for n in kf_frames:
        rgb.append(keyframe_frames(rng, n, q, change))
        p = palettes(rng, n_palettes)
        p[1::2] = p[0::2] ^ rng.integers(0, 2, p[1::2].shape)  # near-identical pairs (Medium tolerance)
        pals.append(p)
        starts.append(starts[-1] + n)
    frame_rgb = np.concatenate(rgb)
    pals = np.stack(pals)
    F = frame_rgb.shape[0]
    kf_of = np.repeat(np.arange(len(kf_frames)), kf_frames)
    dith, palpix = choose_palettes(frame_rgb, pals, kf_of)
    canon, thm, tvm = prepare_tile_mirrors(palpix.reshape(F * q, 64))
    return Video(frame_rgb, np.array(starts, np.int64), pals, np.stack([palette_centroids(p) for p in pals]),
                 canon, thm, tvm, dith.reshape(-1))


def choose_palettes(frame_rgb: np.ndarray, pals: np.ndarray, kf_of: np.ndarray):
    """Stand-in for PrepareDitherTiles' DitheringPalIndex choice (out of scope): per tile, the keyframe palette
    with the lowest total nearest-colour error; also returns that nearest-colour palettisation."""
    F, q = frame_rgb.shape[:2]
    px = frame_rgb.reshape(F, q, 64).astype(np.int64)
    palpix = np.zeros((F, q, 64), np.uint8)
    dith = np.zeros((F, q), np.int32)
    for f in range(F):
        c = pals[kf_of[f]].astype(np.int64)  # [P][16]
        d = np.zeros((q, c.shape[0], 64, c.shape[1]), np.int64)
        for s in (0, 8, 16):
            t = ((px[f] >> s) & 255)[:, None, :, None] - ((c >> s) & 255)[None, :, None, :]
            d += t * t
        best_c = d.argmin(3)                                              # [q][P][64]
        err = np.take_along_axis(d, best_c[..., None], 3)[..., 0].sum(2)  # [q][P]
        pbest = err.argmin(1)
        dith[f] = pbest
        palpix[f] = best_c[np.arange(q), pbest].astype(np.uint8)
    return dith, palpix


def video_from_frames(frames: np.ndarray, kf_of_frame, pals: np.ndarray, ditherer) -> Video:
    """Load -> Dither without synthetic shortcuts for the parts that are built: keyframes from the Load step's
    split (kf_of_frame), every tile dithered by `ditherer(rgb, pal_of, palettes) -> (palpix, hm, vm)` (DitherTile
    Thomas Knoll + PrepareTileMirrors: tiler_amd.dither.dither_tiles, or the oracle's restatement) with the
    keyframe palettes pals[KF][P][16] and the stand-in DitheringPalIndex choice above."""
    frames = np.ascontiguousarray(frames, np.int32)
    F, q = frames.shape[:2]
    kf_of = np.asarray(kf_of_frame, np.int64)
    KF, P = pals.shape[:2]
    dith, _ = choose_palettes(frames, pals, kf_of)
    flat_of = (kf_of[:, None] * P + dith).reshape(-1).astype(np.int32)  # keyframe palettes stacked
    palpix, thm, tvm = ditherer(frames.reshape(-1, 64), flat_of, pals.reshape(KF * P, -1))
    starts = np.r_[np.flatnonzero(np.r_[True, kf_of[1:] != kf_of[:-1]]), F].astype(np.int64)
    return Video(frames, starts, pals, np.stack([palette_centroids(p) for p in pals]), np.asarray(palpix, np.uint8),
                 np.asarray(thm, np.uint8), np.asarray(tvm, np.uint8), dith.reshape(-1))


def video_from_dither(frames: np.ndarray, kf_start, pals: np.ndarray, centroids: np.ndarray, dith: np.ndarray,
                      ditherer) -> Video:
    """Load -> Dither with generated palettes: keyframe palettes pals [KF][P][16], PaletteCentroids [KF][P][192] and
    every tile's DitheringPalIndex dith [F*Q] (tiler_amd.palette.generate_palettes or the oracle's), every tile
    dithered by `ditherer(rgb, pal_of, palettes)` (FinishDitherTiles main.pas:2482-2544)."""
    frames = np.ascontiguousarray(frames, np.int32)
    F, q = frames.shape[:2]
    kf_start = np.asarray(kf_start, np.int64)
    KF, P = pals.shape[:2]
    kf_of = np.repeat(np.arange(KF), np.diff(kf_start))
    dith = np.asarray(dith, np.int32).reshape(F, q)
    flat_of = (kf_of[:, None] * P + dith).reshape(-1).astype(np.int32)
    palpix, thm, tvm = ditherer(frames.reshape(-1, 64), flat_of, np.asarray(pals, np.int32).reshape(KF * P, -1))
    return Video(frames, kf_start, np.asarray(pals, np.int32), np.asarray(centroids, np.float64),
                 np.asarray(palpix, np.uint8), np.asarray(thm, np.uint8), np.asarray(tvm, np.uint8), dith.reshape(-1))


def globaltiling_workload(seed: int, n: int = 1 << 20, protos: int = 65536, noise: float = 0.1,
                          n_palettes: int = 128, zipf: float = 1.1, palsize: int = 16):
    """SURVEY.md 8(d) C4 GlobalTiling input: n palette-index tiles drawn from `protos` prototypes with
    `noise` per-byte perturbation, DitheringPalIndex bins with Zipf(`zipf`) sizes over `n_palettes`."""
    rng = np.random.default_rng(seed)
    P = rng.integers(0, palsize, (protos, 64)).astype(np.uint8)
    tiles = P[rng.integers(0, protos, n)]
    flip = rng.random(tiles.shape) < noise
    tiles[flip] = rng.integers(0, palsize, int(flip.sum())).astype(np.uint8)
    w = 1.0 / np.arange(1, n_palettes + 1) ** zipf
    dith = rng.choice(n_palettes, size=n, p=w / w.sum()).astype(np.int32)
    return tiles, dith

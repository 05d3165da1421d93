"""GlobalTiling step (btnDoGlobalTilingClick main.pas:837-856 -> DoGlobalTiling main.pas:4256-4370).

Host bookkeeping mirrors the reference procedures by name; the K-Modes reduction and the medoid choice
run on the GPU, all palette bins in one batch (tiler_kmodes_batch / tiler_kmodes_medoids_batch; the
reference runs the bins concurrently with ProcThreadPool, main.pas:4339):
  write_tile_dataset_line  WriteTileDatasetLine main.pas:4167-4183 (+ GetTilePalZoneThres 4142-4165)
  equal_quality_tile_count EqualQualityTileCount main.pas:722-725
  do_global_tiling         DoGlobalTiling 4256-4331 + DoKModes 4195-4254 + MergeTiles 3688-3712
  make_tiles_unique        MakeTilesUnique 2555-2612 (stable order: lowest index represents duplicates)
  reindex_tiles            ReindexTiles 4483-4527 (UseCount desc, old index asc)
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import numpy as np

from ._lib import check, load
from .kmodes import compute_kmodes_batch, medoids_batch

CRANDOM_KMODES_COUNT = 7  # cRandomKModesCount main.pas:19


def write_tile_dataset_line(tiles: np.ndarray, palsize: int = 16) -> np.ndarray:
    """[T, 64] palette indices -> [T, 80] K-Modes rows: 64 indices + 16 zone flags
    (count(idx*16 div palsize == z) > palsize div 16)."""
    t = np.asarray(tiles, np.uint8).reshape(-1, 64)
    zone = (t.astype(np.int64) * 16) // palsize
    acc = np.stack([(zone == z).sum(1) for z in range(16)], 1)
    flags = (acc > (palsize // 16)).astype(np.uint8)
    return np.ascontiguousarray(np.concatenate([t, flags], 1))


FPC_INV_LN2 = 1.4426950408889634079  # FPC Math.log2(x) = ln(x) * 1.4426950408889634079


def equal_quality_tile_count(n: float) -> int:
    """round(sqrt(n) * log2(1 + n)) (main.pas:722-725) with FPC's banker's rounding (Python round is half-even)
    and FPC Math's log2 = ln(x) * (1 / ln 2)."""
    return int(round(math.sqrt(n) * (math.log(1.0 + n) * FPC_INV_LN2)))


def kmodes_medoids(X: np.ndarray, labels: np.ndarray, centroids: np.ndarray):
    lib = load()
    X = np.ascontiguousarray(X, np.uint8)
    labels = np.ascontiguousarray(labels, np.int32)
    centroids = np.ascontiguousarray(centroids, np.uint8)
    k = centroids.shape[0]
    medoid = np.zeros(k, np.int32)
    counts = np.zeros(k, np.int32)
    v = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    check(lib.tiler_kmodes_medoids(v(X), X.shape[0], v(labels), v(centroids), k, v(medoid), v(counts)),
          "tiler_kmodes_medoids")
    return medoid, counts


def merge_tiles(idx, best, palpix, active, use_count, merge_index):
    """MergeTiles main.pas:3688-3712 (NewTile = nil)."""
    for j in idx:
        if j == best:
            continue
        use_count[best] += use_count[j]
        active[j] = 0
        merge_index[j] = best
        palpix[j] = 0


@dataclass
class GTPlan:
    """DoGlobalTiling's binning (main.pas:4272-4331): the K-Modes rows, the active tiles of each palette bin,
    their StartingPoint and ClusterCount, and the bins that go through K-Modes (`run`)."""
    lines: np.ndarray
    bins: list
    starts: list
    k_per_bin: np.ndarray
    run: list


def plan_global_tiling(palpix, dith_pal, n_palettes: int, desired: int, palsize: int = 16,
                       restart: int = CRANDOM_KMODES_COUNT, active=None) -> GTPlan:
    palpix = np.asarray(palpix, np.uint8).reshape(-1, 64)
    T = palpix.shape[0]
    active = np.ones(T, np.uint8) if active is None else np.asarray(active, np.uint8)
    dith_pal = np.asarray(dith_pal, np.int64)
    lines = write_tile_dataset_line(palpix, palsize)
    act = np.nonzero(active)[0]
    bins = [act[dith_pal[act] == p] for p in range(n_palettes)]
    # StartingPoint: last row of the bin with minimal byte sum (acc <= best), -restart when empty
    starts = []
    for b in bins:
        if b.size == 0:
            starts.append(-restart)
            continue
        s = lines[b].astype(np.int64).sum(1)
        starts.append(int(b.size - 1 - np.argmin(s[::-1])))
    dis_cnt = sum(equal_quality_tile_count(b.size) for b in bins)
    share = desired / dis_cnt
    k_per_bin = np.zeros(n_palettes, np.int64)
    run = []  # bins that go through K-Modes (DoKModes, main.pas:4195-4254)
    for p, b in enumerate(bins):
        kc = math.ceil(equal_quality_tile_count(b.size) * share)
        k_per_bin[p] = int(round(kc))
        if b.size > kc:
            run.append(p)
    return GTPlan(lines, bins, starts, k_per_bin, run)


def kmodes_bins(plan: GTPlan, subset, palsize: int = 16) -> dict:
    """K-Modes + medoids of the listed bins in ONE GPU batch: {bin: (labels, medoid, counts)}, bin-local."""
    subset = list(subset)
    if not subset:
        return {}
    X = np.ascontiguousarray(np.concatenate([plan.lines[plan.bins[p]] for p in subset]))
    off = np.zeros(len(subset) + 1, np.int32)
    off[1:] = np.cumsum([plan.bins[p].size for p in subset])
    ks = np.array([plan.k_per_bin[p] for p in subset], np.int32)
    st = np.array([plan.starts[p] for p in subset], np.int32)
    labels, cent, _, _ = compute_kmodes_batch(X, off, ks, st, palsize)
    medoid, counts = medoids_batch(X, off, ks, labels, cent)
    koff = np.concatenate([[0], np.cumsum(ks)])
    return {p: (labels[off[i]:off[i + 1]], medoid[koff[i]:koff[i + 1]], counts[koff[i]:koff[i + 1]])
            for i, p in enumerate(subset)}


def kmodes_merge_map(plan: GTPlan, results: dict, T: int) -> np.ndarray:
    """DoKModes' merge decisions (main.pas:4231-4253) of the bins in `results` as one int32 map over all T tiles:
    merge_to[j] = the medoid tile j merges into, -1 = kept.  Bins own disjoint tiles, so maps of different bin
    sets combine with an element-wise max (the sharded path's all-reduce)."""
    merge_to = np.full(T, -1, np.int32)
    for p, (labels, medoid, counts) in results.items():
        b = plan.bins[p]
        best = np.where(counts >= 2, b[np.maximum(medoid, 0)], -1)[labels]
        sel = (best >= 0) & (b != best)
        merge_to[b[sel]] = best[sel]
    return merge_to


def apply_merge_map(merge_to, palpix, active, use_count):
    """MergeTiles for every merged tile (main.pas:3688-3712, NewTile = nil): UseCount summed into the medoid,
    Active := False, MergeIndex set, PalPixels zeroed.  Each medoid is kept (merge_to = -1), so the order of the
    reference's per-cluster loop does not change the result."""
    palpix = np.array(palpix, np.uint8, copy=True).reshape(-1, 64)
    T = palpix.shape[0]
    active = np.ones(T, np.uint8) if active is None else np.array(active, np.uint8, copy=True)
    use_count = np.ones(T, np.int64) if use_count is None else np.array(use_count, np.int64, copy=True)
    merge_to = np.asarray(merge_to, np.int64)
    src = np.nonzero(merge_to >= 0)[0]
    dst = merge_to[src]
    np.add.at(use_count, dst, use_count[src])
    active[src] = 0
    merge_index = np.full(T, -1, np.int64)
    merge_index[src] = dst
    palpix[src] = 0
    return palpix, active, use_count, merge_index


def apply_kmodes_merges(plan: GTPlan, results: dict, palpix, active, use_count):
    """MergeTiles for every cluster with >= 2 members (main.pas:4231-4253) of every K-Modes bin."""
    T = np.asarray(palpix).reshape(-1, 64).shape[0]
    return apply_merge_map(kmodes_merge_map(plan, results, T), palpix, active, use_count)


def do_global_tiling(palpix, dith_pal, n_palettes: int, desired: int, palsize: int = 16,
                     restart: int = CRANDOM_KMODES_COUNT, active=None, use_count=None):
    """Returns (palpix, active, use_count, merge_index, k_per_bin) after the K-Modes merge pass
    (the caller applies merge_index to tilemaps: FinishMergeTiles main.pas:3722-3734)."""
    plan = plan_global_tiling(palpix, dith_pal, n_palettes, desired, palsize, restart, active)
    res = kmodes_bins(plan, plan.run, palsize)
    pp, act, uc, mi = apply_kmodes_merges(plan, res, palpix, active, use_count)
    return pp, act, uc, mi, plan.k_per_bin


def make_tiles_unique(palpix, active, use_count):
    """MakeTilesUnique main.pas:2555-2612 over all tiles.  Active tiles sorted by CompareTilePalPixels
    (CompareDWord over 16 little-endian dwords, main.pas:2546-2553; equal keys by index: TFPList.Sort is
    unstable); each run of identical tiles merges into its first member.  The final
    DoOneMerge runs with i = Count - 1 (main.pas:2604-2605), so the last run never includes its last member
    and a 2-member last run does not merge: reproduced, not fixed."""
    palpix = np.array(palpix, np.uint8, copy=True)
    active = np.array(active, np.uint8, copy=True)
    use_count = np.array(use_count, np.int64, copy=True)
    merge_index = np.full(palpix.shape[0], -1, np.int64)
    idx = np.nonzero(active)[0]
    if idx.size:
        words = np.ascontiguousarray(palpix[idx]).view("<u4").reshape(-1, 16)
        order = idx[np.lexsort(words[:, ::-1].T)]  # dword 0 primary; stable: index order among equal keys
        w = np.ascontiguousarray(palpix[order]).view("<u4").reshape(-1, 16)
        starts = np.concatenate([[0], np.nonzero(np.any(w[1:] != w[:-1], axis=1))[0] + 1])
        ends = np.concatenate([starts[1:], [order.size]])
        ends[-1] -= 1  # the reference's final DoOneMerge: i := sortList.Count - 1
        for a, b in zip(starts, ends):
            if b - a >= 2:
                members = order[a:b]
                merge_tiles(members, int(members[0]), palpix, active, use_count, merge_index)
    return palpix, active, use_count, merge_index


def reindex_tiles(active, use_count):
    """ReindexTiles main.pas:4483-4527: idx_map[old] = new, order (UseCount desc, old index asc)."""
    act = np.nonzero(active)[0]
    order = act[np.lexsort((act, -np.asarray(use_count)[act]))]
    idx_map = np.full(np.asarray(active).shape[0], -1, np.int64)
    idx_map[order] = np.arange(order.size)
    return idx_map

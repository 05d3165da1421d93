"""BASELINE C4 end to end at size: 1080p GlobalTiling of ~1M tiles -> 64k, then FrameTiling of a
keyframe against the REDUCED tileset's real candidate set, through tiler_amd.encoder's steps (main.pas:1232-1272:
MakeUnique -> GlobalTiling = K-Modes merges + MakeTilesUnique + ReindexTiles (main.pas:4256-4370, 4483-4527) ->
FrameTiling).  Each link is checked against the CPU restatement where the restatement finishes in seconds:

* K-Modes: every palette bin of <= 3,000 rows re-run by oracle/tiler_oracle.c (labels, centroids, medoids) and its
  merge-map entries (DoKModes main.pas:4231-4253) compared tile by tile;
* MakeTilesUnique + ReindexTiles at full size: oracle.make_tiles_unique / oracle.reindex over the GPU-merged tileset
  give the encoder's tileset, Active, UseCount and remapped TileMap items;
* PrepareFrameTiling: 1,000 sampled items' k = 8 searches against the restated ANN search (the used table itself is
  the host UseOne over the GPU's k = 8 results of every item);
* DoFrameTiling: 1,500 sampled frame tiles of the keyframe against the restated ANN search over the same
  candidate set -- tile, palette, mirror flags and fp32 error bit for bit.

Input: the C4 GlobalTiling workload (synth.globaltiling_workload: 64k prototypes, 10 % perturbation, Zipf bins over
128 palettes) laid out as 33 frames of 1080p; frame tiles are the tiles rendered in their palette and original
orientation; keyframe 0 is the first 3 frames (97,200 tiles; FrameTiling of a 24-frame keyframe is bench.py's)."""
import numpy as np
import pytest

from tiler_amd import synth

pytestmark = pytest.mark.gpu

Q = 32400  # 1080p, 8x8 tiles
F = 33     # 1,069,200 tiles
P = 128


def _render(palpix, hm, vm, dith, pals):
    """RGB frame tiles: the palette-index tile in its ORIGINAL orientation (undo PrepareTileMirrors) in its palette."""
    t = palpix.copy()
    h = hm.astype(bool)
    v = vm.astype(bool)
    t[v] = synth.vflip(t[v])  # prepare_tile_mirrors applied hflip then vflip: undo in reverse order
    t[h] = synth.hflip(t[h])
    return pals[dith[:, None], t.astype(np.int64)].astype(np.int32)


@pytest.mark.timeout(900)
def test_c4_chain_at_size(gpu, oracle):
    from tiler_amd import frame_tiling as ftm
    from tiler_amd import global_tiling as gt
    from tiler_amd.encoder import Encoder
    rng = np.random.default_rng(44)
    raw, dith = synth.globaltiling_workload(4, F * Q, n_palettes=P)
    palpix, hm, vm = synth.prepare_tile_mirrors(raw)
    pals = synth.palettes(rng, P)
    cents = synth.palette_centroids(pals)
    frames = _render(palpix, hm, vm, dith, pals).reshape(F, Q, 64)
    kf_start = np.array([0, 3, F])
    v = synth.Video(frames, kf_start, np.stack([pals, pals]), np.stack([cents, cents]), palpix, hm, vm, dith)
    e = Encoder(v, frames=np.arange(3))  # keyframe 0's frames and tilemaps; the tileset is the whole clip's
    e.do_make_unique()
    pp0, act0, uc0 = e.palpix.copy(), e.active.copy(), e.use_count.copy()

    # ---- GlobalTiling: K-Modes of every bin in one GPU batch, merge map checked on the small bins ----
    plan = gt.plan_global_tiling(pp0, e.dith_pal, P, 65536, active=act0)
    assert int(act0.sum()) > 1_000_000 and len(plan.run) > 100
    res = gt.kmodes_bins(plan, plan.run)
    T = pp0.shape[0]
    merge_to = gt.kmodes_merge_map(plan, res, T)
    small = [p for p in plan.run if plan.bins[p].size <= 3000]
    assert len(small) >= 40
    checked = 0
    for p in small:
        b = plan.bins[p]
        X = plan.lines[b]
        k = int(plan.k_per_bin[p])
        ol, oc, _, _ = oracle.kmodes(X, k, plan.starts[p], threads=16)
        labels, medoid, counts = res[p]
        assert np.array_equal(labels, ol), p
        omed = np.full(k, -1, np.int64)
        for j in np.nonzero(np.bincount(ol, minlength=k))[0]:
            mem = np.nonzero(ol == j)[0]
            i, _ = oracle.km_get_min(X[mem], oc[j])
            omed[j] = mem[i]
        ocnt = np.bincount(ol, minlength=k)
        best = np.where(ocnt >= 2, b[np.maximum(omed, 0)], -1)[ol]
        want = np.where((best >= 0) & (b != best), best, -1)
        assert np.array_equal(merge_to[b], want), p
        checked += b.size
    assert checked > 20000
    pp, act, uc, mi = gt.apply_merge_map(merge_to, pp0, act0, uc0)
    e.palpix, e.active, e.use_count = pp, act, uc
    e.finish_merge_tiles(mi)
    tile_before = e.tile.copy()
    # MakeTilesUnique over all tiles + ReindexTiles, restated on the same merged tileset
    e.make_tiles_unique()
    opp, oact, ouc, omi = oracle.make_tiles_unique(pp, act, uc)
    assert np.array_equal(e.palpix, opp) and np.array_equal(e.active, oact) and np.array_equal(e.use_count, ouc)
    remap = np.asarray(omi)[tile_before]
    assert np.array_equal(e.tile, np.where(remap >= 0, remap, tile_before))
    oidx = oracle.reindex(oact, ouc)
    e.reindex_tiles()
    assert np.array_equal(e.tile, oidx[np.where(remap >= 0, remap, tile_before)])
    key = np.where(oidx >= 0, oidx.astype(np.int64), np.iinfo(np.int64).max)
    order = np.argsort(key, kind="stable")[: int((oidx >= 0).sum())]
    assert np.array_equal(e.palpix, opp[order]) and np.array_equal(e.use_count, ouc[order])
    assert 60000 <= e.palpix.shape[0] <= 70000  # 1M -> the desired 64k (+ bins below their K)

    # ---- FrameTiling of keyframe 0 against the reduced tileset's candidate set ----
    items_t, items_p = e.tile[0:3].ravel().copy(), e.pal[0:3].ravel().copy()
    errs = e.do_frame_tiling(ftm.FT_MEDIUM)
    assert np.isfinite(errs).all()
    # k = 8 preselection of sampled items vs the restated ANN search (PrepareGlobalFT rows of the reduced set)
    gds = ftm.prepare_global_ft(e.palpix, e.active)
    keys = np.unique(items_p.astype(np.int64) * e.palpix.shape[0] + items_t)
    ks = np.random.default_rng(4).choice(keys, min(1000, keys.size), replace=False)
    qk = e.palpix[ks % e.palpix.shape[0]].astype(np.float32)
    gi8, ge8 = gds.kdt.search_batch(qk, k=8)
    corr, hi = ftm.palette_corr(cents)
    used = ftm.mark_used(gds, e.palpix, items_p, items_t, P, ftm.FT_MEDIUM, corr, hi)
    gds.kdt.close()
    o_ds, _, _ = oracle.prepare_global_ds(e.palpix, e.active)
    okd = oracle.KDTree(o_ds)
    oi8, oe8 = okd.search_batch(qk, k=8)
    okd.close()
    assert np.array_equal(gi8, oi8) and np.array_equal(ge8.view(np.uint32), oe8.view(np.uint32))
    # sampled frame tiles vs the restated search over the same candidate set
    ods, ot, op, oa = oracle.build_ft_dataset(used, e.palpix, e.thm, e.tvm, pals)
    assert ods.shape[0] > 10000
    pick = np.random.default_rng(5).choice(3 * Q, 1500, replace=False)
    o = oracle.frame_tiling(frames[0:3].reshape(-1, 64)[pick], ods, ot, op, oa)
    # FrameTiling ran last: e.tile / e.pal / e.hm / e.vm hold its tilemap items
    assert np.array_equal(e.tile.ravel()[pick], o[0])
    assert np.array_equal(e.pal.ravel()[pick], o[1])
    assert np.array_equal(e.hm.ravel()[pick], o[2]) and np.array_equal(e.vm.ravel()[pick], o[3])
    assert np.array_equal(errs.ravel()[pick].view(np.uint32), o[4].view(np.uint32))

"""Debug helper (GPU box): replay test_pipeline's chain up to FrameTiling and localise a GPU/oracle difference:
the k=8 preselection (used table) or the k=1 FrameTiling search of the keyframe dataset."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as oracle  # noqa: E402
from test_pipeline import _OracleChain  # noqa: E402

import tiler_amd  # noqa: E402
from tiler_amd import frame_tiling as ft  # noqa: E402
from tiler_amd import synth  # noqa: E402
from tiler_amd.encoder import Encoder  # noqa: E402

tiler_amd.load().tiler_init(0)
quality = int(sys.argv[1]) if len(sys.argv) > 1 else 1
v = synth.video(51 + quality, 320, 240, kf_frames=(3, 3), n_palettes=8)
e = Encoder(v)
e.do_make_unique()
e.do_global_tiling(700)
o = _OracleChain(v)
T0, Q = o.palpix.shape[0], v.tiles_per_frame
gds = ft.prepare_global_ft(e.palpix, e.active)
ogds, ogt, oga = oracle.prepare_global_ds(e.palpix)
print("T", e.palpix.shape[0], "gds rows", ogds.shape[0])
# k=8 search itself
keys = np.unique(np.asarray(e.pal, np.int64) * e.palpix.shape[0] + np.asarray(e.tile, np.int64))
til = keys % e.palpix.shape[0]
qs = e.palpix[til].astype(np.float32)
gi, ge = gds.kdt.search_batch(qs, k=8)
okd = oracle.KDTree(ogds)
oi, oe = okd.search_batch(qs, k=8)
print("k8 pos equal:", np.array_equal(gds.kdt.positions(), okd.positions()))
bad = np.nonzero(np.any(gi != oi, 1))[0]
print("k8 queries", qs.shape[0], "differ", bad.size, "dist differ", int(np.count_nonzero(ge != oe)))
for b in bad[:5]:
    print(b, gi[b], ge[b], "|", oi[b], oe[b])
print("gds stats", gds.kdt.stats())
for k in range(v.kf_start.size - 1):
    f0, f1 = int(v.kf_start[k]), int(v.kf_start[k + 1])
    corr, hi = oracle.palette_corr(v.centroids[k])
    ug = ft.mark_used(gds, e.palpix, e.pal[f0:f1].ravel(), e.tile[f0:f1].ravel(), v.palettes.shape[1], quality,
                      *ft.palette_corr(v.centroids[k]))
    uo = oracle.mark_used(ogds, ogt, oga, e.pal[f0:f1].ravel(), e.tile[f0:f1].ravel(), e.palpix, v.palettes.shape[1],
                          quality, corr, hi)
    print("kf", k, "used equal:", np.array_equal(ug, uo), int(ug.sum()), int(uo.sum()))
    ds, ti, pi, at = oracle.build_ft_dataset(uo, e.palpix, e.thm, e.tvm, v.palettes[k])
    kt = ft.KeyframeTiler(e.palpix, e.thm, e.tvm, v.palettes[k], synth.ft_dataset_from_used(uo, e.thm, e.tvm))
    g = kt.do_frame_tiling(v.frame_rgb[f0:f1])
    st = kt.kdt.stats()
    kt.finish_frame_tiling()
    r = oracle.frame_tiling(v.frame_rgb[f0:f1], ds, ti, pi, at)
    d = np.nonzero((g[0] != r[0]) | (g[1] != r[1]) | (g[2] != r[2]) | (g[3] != r[3]))[0]
    print("kf", k, "FT items differ", d.size, "of", g[0].size, "err differ", int(np.count_nonzero(g[4] != r[4])),
          st)
    rows = kt.rows if hasattr(kt, "rows") else None
    for j in d[:5]:
        print("  q", j, "gpu", g[0][j], g[1][j], g[2][j], g[3][j], g[4][j], "oracle", r[0][j], r[1][j], r[2][j], r[3][j],
              r[4][j])

#!/usr/bin/env python3
"""Study script: ann_kdtree_pri_search on the GPU (kd_pri_kernel, the priority search replayed one thread per
query) -- lone-call latency and batched rate on the C3 keyframe handle (262,144 PsyV rows of a tileset in 4
orientations) and on a 12,000-row handle, frame-tile queries; answers checked against ann_kdtree_search's distance
(eps = 0: the same exact minimum)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import tiler_amd
    from tiler_amd import synth
    rng = np.random.default_rng(12)
    P, T = 128, 65536
    pals = synth.palettes(rng, P)
    tiles, thm, tvm = synth.tileset(rng, T)
    ds = synth.ft_dataset_from_used(synth.used_one_palette(rng.integers(0, P, T).astype(np.int32), P), thm, tvm)
    rows = tiler_amd.psyv_batch(palpix=tiles, tile_of=ds.tile_of, palettes=pals, pal_of=ds.pal_of,
                                flags_per=ds.psyv_flags, flags=1 | 2, gamma=-1, want32=True)[1]
    wl = synth.make_workload(13, 1920, 1080, 1, 256, n_palettes=8)
    _, qd = tiler_amd.psyv_batch(rgb=wl.frame_rgb[0].reshape(-1, 64)[:1024], flags=2, want64=False, want32=True)
    qd = np.ascontiguousarray(qd, np.float32)
    out = {}
    for name, data in (("c3_262144", rows), ("small_12000", rows[rng.choice(rows.shape[0], 12000, replace=False)])):
        with tiler_amd.KDTree(data) as kdt:
            si, se = kdt.search_batch(qd)
            kdt.pri_search(qd[0])
            lat = []
            for i in range(8):
                t0 = time.perf_counter()
                kdt.pri_search(qd[i])
                lat.append(time.perf_counter() - t0)
            slow = []
            for i in range(64):  # lone calls: which queries take the replay (> 5 ms)
                t0 = time.perf_counter()
                kdt.pri_search(qd[i])
                if time.perf_counter() - t0 > 5e-3:
                    slow.append(i)
            t0 = time.perf_counter()
            pi, pe = kdt.pri_search_batch(qd)
            dt = time.perf_counter() - t0
            out[name] = {"lone_ms_median": round(1e3 * float(np.median(lat)), 3), "batch_queries": len(qd),
                         "batch_queries_per_s": round(len(qd) / dt, 1),
                         "dist_equal_std": int(np.count_nonzero(pe.view(np.uint32) == se.view(np.uint32))),
                         "idx_differ_std": int(np.count_nonzero(pi != si)),
                         "replayed_of_first_64": len(slow), "replayed_ids": slow[:16],
                         "ties_within_std_dist": [int(np.count_nonzero(np.sum((data - qd[i]) ** 2, 1) <= se[i] * (1 + 1e-6)))
                                                  for i in slow[:8]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

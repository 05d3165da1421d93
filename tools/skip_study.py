"""Design study (CPU): how often can the orbit shortlist skip isotypic blocks x = 1..3 of a (query block,
tile block) pair after computing d_0 alone?

Per lane (one query, 16 tiles of a 32-tile block) the shortlist bound of tile t is
    u_t = d0_t - |c_t|^2/2 + |d1_t| + |d2_t| + |d3_t|,   d_x = (P_x q).(P_x c_t)
and Cauchy-Schwarz gives the cheap lane bound
    u_t <= max_t (d0_t - |c_t|^2/2) + sum_x |P_x q| * max_t |P_x c_t|.
A lane whose cheap bound is <= its list threshold (the L-th best sub-block bound so far) cannot insert
anything from this block; a query block (32 queries, 64 lanes) skips x = 1..3 when every lane can.
Simulates the kernel's scan (L = 4 sub-blocks of 4 tiles per lane) in fp64 on the C3 workload and
prints the share of (query block, tile block) pairs that still need the full contraction.

    python tools/skip_study.py [n_query_blocks] [order]      order: index | dc
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import pyoracle as oracle  # noqa: E402
from tiler_amd import synth  # noqa: E402
from tools.prune_study import projections  # noqa: E402


def main(nqb=6, order="index", seed=7, T=65536, L=4):
    wl = synth.make_workload(seed, 1920, 1080, 1, T, n_palettes=128)
    used = synth.used_one_palette(wl.tile_pal, 128)
    rows, *_ = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    base = rows[0::4].astype(np.float64)  # one group per tile (all 4 orientations present)
    if order == "dc":
        base = base[np.argsort(base[:, 0], kind="stable")]
    G = base.shape[0]
    P = projections()
    cx = [base @ P[x].T for x in range(4)]
    cn = np.stack([np.linalg.norm(c, axis=1) for c in cx], 1)  # [G][4]
    seed_c = -0.5 * (base ** 2).sum(1)
    q_all = oracle.psyv_batch(wl.tiles_per_frame, rgb=wl.frame_rgb[0], flags=2).astype(np.float64)
    rng = np.random.default_rng(3)
    nblk = G // 32
    # lane layout of one 32x32 accumulator block: lane (j, h) holds tiles 8 s + 4 h + i, s, i in 0..3
    tiles_of_h = [np.array([8 * s + 4 * h + i for s in range(4) for i in range(4)]) for h in (0, 1)]
    need_tot, n_tot = 0, 0
    for qb in rng.choice(q_all.shape[0] // 32, nqb, replace=False):
        q = q_all[qb * 32:(qb + 1) * 32]
        qx = [q @ P[x].T for x in range(4)]
        qn = np.stack([np.linalg.norm(v, axis=1) for v in qx], 1)  # [32][4]
        d = [qx[x] @ cx[x].T for x in range(4)]  # [32][G]
        u = d[0] + seed_c[None] + np.abs(d[1]) + np.abs(d[2]) + np.abs(d[3])
        d0s = d[0] + seed_c[None]
        lists = np.full((2, 32, L), -np.inf)  # best sub-block bounds per lane, descending
        need = np.zeros(nblk, bool)
        lane_need = []
        for b in range(nblk):
            g0 = b * 32
            for h in (0, 1):
                tt = g0 + tiles_of_h[h]
                Mx = cn[tt].max(0)  # [4]
                cheap = d0s[:, tt].max(1) + (qn[:, 1:] * Mx[None, 1:]).sum(1)
                thr = lists[h][:, L - 1]
                if np.any(cheap > thr):
                    need[b] = True
                lane_need.append(np.mean(cheap > thr))
                sb = u[:, tt].reshape(32, 4, 4).max(2)  # [32][4 sub-blocks]
                allv = np.concatenate([lists[h], sb], 1)
                lists[h] = -np.sort(-allv, 1)[:, :L]
        print("per-lane share of blocks with cheap bound above the threshold: %.3f (last half %.3f)"
              % (np.mean(lane_need), np.mean(lane_need[len(lane_need) // 2:])))
        print("query block %6d: full contraction needed for %.3f of %d tile blocks (first 256: %.3f, last 1024: %.3f)"
              % (qb, need.mean(), nblk, need[:256].mean(), need[-1024:].mean()), flush=True)
        need_tot += need.sum()
        n_tot += nblk
    print("order=%s: overall %.3f" % (order, need_tot / n_tot))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 6, sys.argv[2] if len(sys.argv) > 2 else "index")

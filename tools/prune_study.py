"""Design study (CPU, oracle as checker): how much of the FrameTiling candidate set an exact,
mirror-invariant lower bound can rule out.  For a tile c and query q with isotypic projections P_x
(the 4 joint eigenspaces of the H/V mirror operators on the Haar descriptor):
    min_m |q - S_m c|^2 >= |P0 q - P0 c|^2 + sum_{x>=1} (|P_x q| - |P_x c|)^2     (LB)
Prints, for sampled frame tiles of the C3 workload, the share of tiles with LB <= the exact NN distance
(the tiles a perfect per-tile filter must still score)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import pyoracle as oracle  # noqa: E402
from tiler_amd import synth  # noqa: E402


def haar_matrix():
    f = 1.0 / np.sqrt(2.0)
    T = np.zeros((64, 64))
    for i in range(64):
        o = np.zeros((8, 8))
        o.flat[i] = 1.0
        n = 8
        while n >= 2:
            blk = o[:n, :n]
            h = n // 2
            tx = np.empty_like(blk)
            tx[:, :h] = (blk[:, 0::2] + blk[:, 1::2]) * f
            tx[:, h:] = (blk[:, 0::2] - blk[:, 1::2]) * f
            ty = np.empty_like(blk)
            ty[:h, :] = (tx[0::2, :] + tx[1::2, :]) * f
            ty[h:, :] = (tx[0::2, :] - tx[1::2, :]) * f
            o[:n, :n] = ty
            n //= 2
        T[:, i] = o.reshape(64)
    return T


def projections():
    T = haar_matrix()
    idx = np.arange(64).reshape(8, 8)
    MH = np.eye(64)[idx[:, ::-1].reshape(64)]
    MV = np.eye(64)[idx[::-1, :].reshape(64)]
    SH = np.kron(np.eye(3), T @ MH @ T.T)
    SV = np.kron(np.eye(3), T @ MV @ T.T)
    I = np.eye(192)
    P = []
    for x in range(4):
        sh = -1.0 if x & 1 else 1.0
        sv = -1.0 if x & 2 else 1.0
        P.append((I + sh * SH) @ (I + sv * SV) / 4.0)
    return P


def main(seed=7, nq=600, T=65536):
    t0 = time.time()
    wl = synth.make_workload(seed, 1920, 1080, 1, T, n_palettes=128)
    used = synth.used_one_palette(wl.tile_pal, 128)
    rows, *_ = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    print("rows", rows.shape, round(time.time() - t0, 1), "s", flush=True)
    rng = np.random.default_rng(1)
    pick = rng.choice(wl.tiles_per_frame, nq, replace=False)
    q = oracle.psyv_batch(nq, rgb=wl.frame_rgb[0][pick], flags=2).astype(np.float32)
    t0 = time.time()
    ni, nd = oracle.nn_batch(rows, q)
    print("nn", round(time.time() - t0, 1), "s", flush=True)
    P = projections()
    print("block ranks", [int(round(np.trace(p))) for p in P])
    base = rows[0::4].astype(np.float64)  # every tile in 4 orientations: base = unmirrored row
    q64 = q.astype(np.float64)
    fc0 = base @ P[0].T
    nc = np.stack([np.linalg.norm(base @ P[x].T, axis=1) for x in (1, 2, 3)], 1)
    fq0 = q64 @ P[0].T
    nqn = np.stack([np.linalg.norm(q64 @ P[x].T, axis=1) for x in (1, 2, 3)], 1)
    share, share_dc = [], []
    for i in range(nq):
        lb = ((fc0 - fq0[i]) ** 2).sum(1) + ((nc - nqn[i]) ** 2).sum(1)
        share.append(np.mean(lb <= nd[i]))
        dc = sum((base[:, 64 * p] - q64[i, 64 * p]) ** 2 for p in range(3))
        share_dc.append(np.mean(dc <= nd[i]))
    share = np.array(share)
    print("LB survivors per query: mean %.4f  median %.4f  p90 %.4f  max %.4f" %
          (share.mean(), np.median(share), np.quantile(share, 0.9), share.max()))
    share_dc = np.array(share_dc)
    print("DC-only survivors: mean %.4f median %.4f" % (share_dc.mean(), np.median(share_dc)))
    e0 = np.mean([np.sum((base @ P[x].T) ** 2) for x in range(4)])
    print("energy share per block (tiles):", [round(float(np.sum((base[:2000] @ P[x].T) ** 2) /
                                                      np.sum(base[:2000] ** 2)), 3) for x in range(4)], e0 > 0)



def pca_blocks(X, leaf):
    """Recursive bisection at the median of the principal axis down to `leaf`-sized blocks:
    returns a permutation whose consecutive `leaf` entries form one block."""
    out = []
    stack = [np.arange(X.shape[0])]
    while stack:
        ix = stack.pop()
        if ix.size <= leaf:
            out.append(ix)
            continue
        Y = X[ix] - X[ix].mean(0)
        # power iteration for the top principal axis
        v = np.random.default_rng(ix.size).normal(size=X.shape[1])
        for _ in range(8):
            v = Y.T @ (Y @ v)
            v /= np.linalg.norm(v) + 1e-30
        p = Y @ v
        o = np.argsort(p, kind="stable")
        h = ((ix.size // leaf + 1) // 2) * leaf if ix.size > 2 * leaf else ix.size // 2
        stack.append(ix[o[h:]])
        stack.append(ix[o[:h]])
    return np.concatenate(out)


def block_study(seed=7, T=65536, qblocks=24, qleaf=64, tleaf=32):
    wl = synth.make_workload(seed, 1920, 1080, 1, T, n_palettes=128)
    used = synth.used_one_palette(wl.tile_pal, 128)
    rows, *_ = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    P = projections()
    feat = lambda X: np.concatenate([X @ P[0].T, np.stack([np.linalg.norm(X @ P[x].T, axis=1) for x in (1, 2, 3)], 1)], 1)  # noqa
    base = rows[0::4].astype(np.float64)
    fc = feat(base)
    # the 192-d P0 part has rank 48: use an orthonormal basis for it
    w, V = np.linalg.eigh(P[0])
    B0 = V[:, w > 0.5]
    fcr = np.concatenate([base @ B0, fc[:, 192:]], 1)
    q_all = oracle.psyv_batch(wl.tiles_per_frame, rgb=wl.frame_rgb[0], flags=2)
    fq = np.concatenate([q_all @ B0, np.stack([np.linalg.norm(q_all @ P[x].T, axis=1) for x in (1, 2, 3)], 1)], 1)
    t0 = time.time()
    tperm = pca_blocks(fcr, tleaf)
    qperm = pca_blocks(fq, qleaf)
    print("blocking", round(time.time() - t0, 1), "s")
    nb = T // tleaf
    rng = np.random.default_rng(2)
    sel = rng.choice(len(qperm) // qleaf, qblocks, replace=False)
    need, need_rand, ball = [], [], []
    rperm = rng.permutation(T)
    for b in sel:
        qi = qperm[b * qleaf:(b + 1) * qleaf]
        q = q_all[qi].astype(np.float32)
        _, nd = oracle.nn_batch(rows, q)
        lb = ((fq[qi][:, None, :] - fcr[None, :, :]) ** 2).sum(2)  # [qleaf][T]
        surv = lb <= nd[:, None].astype(np.float64) * (1 + 1e-6)
        anyb = surv[:, tperm].reshape(qleaf, nb, tleaf).any(2).any(0)
        need.append(anyb.mean())
        need_rand.append(surv[:, rperm].reshape(qleaf, nb, tleaf).any(2).any(0).mean())
        # ball bound per (query, tile block): centre = block mean, radius = max member distance
        fb = fcr[tperm].reshape(nb, tleaf, -1)
        mu = fb.mean(1)
        rad = np.sqrt(((fb - mu[:, None, :]) ** 2).sum(2)).max(1)
        dq = np.sqrt(((fq[qi][:, None, :] - mu[None]) ** 2).sum(2))
        lbb = np.maximum(dq - rad[None], 0) ** 2
        ball.append((lbb <= nd[:, None]).any(0).mean())
    need = np.array(need)
    print("tile blocks needed per %d-query block (PCA blocks): mean %.4f median %.4f max %.4f; random blocks %.4f"
          % (qleaf, need.mean(), np.median(need), need.max(), np.mean(need_rand)))
    print("ball bound per (query, tile block): mean %.4f median %.4f" % (np.mean(ball), np.median(ball)))




def ivf_study(seed=7, T=65536, C=256, wgs=6, wg=512, wave=64, tblk=32):
    """IVF-style scheme: tiles ordered by coarse cluster, queries sorted by nearest cluster, WG of `wg`
    queries; threshold T_q = best exact distance within the query's own cluster; a (wave, tile block)
    pair is needed if any pair has LB <= T_q."""
    wl = synth.make_workload(seed, 1920, 1080, 1, T, n_palettes=128)
    used = synth.used_one_palette(wl.tile_pal, 128)
    rows, *_ = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    P = projections()
    w, V = np.linalg.eigh(P[0])
    B0 = V[:, w > 0.5]
    feat = lambda X: np.concatenate([X @ B0, np.stack([np.linalg.norm(X @ P[x].T, axis=1) for x in (1, 2, 3)], 1)], 1)  # noqa
    base = rows[0::4].astype(np.float64)
    fc = feat(base)
    leaf = T // C
    tperm = pca_blocks(fc, leaf)
    cl_of = np.empty(T, np.int64)
    cl_of[tperm] = np.arange(T) // leaf
    cent = np.stack([fc[tperm[i * leaf:(i + 1) * leaf]].mean(0) for i in range(C)])
    q_all = oracle.psyv_batch(wl.tiles_per_frame, rgb=wl.frame_rgb[0], flags=2)
    fq = feat(q_all)
    qc = (((fq[:, None, :] - cent[None]) ** 2).sum(2)).argmin(1)
    qord = np.argsort(qc, kind="stable")
    rng = np.random.default_rng(3)
    starts = rng.choice(len(qord) // wg, wgs, replace=False) * wg
    r4 = rows.astype(np.float64).reshape(T, 4, 192)
    nc2 = (r4 ** 2).sum(2)  # [T][4]
    frac, frac_wg, frac_dstar = [], [], []
    for s in starts:
        qi = qord[s:s + wg]
        q = q_all[qi]
        # exact min over mirrors of distances to own-cluster tiles -> T_q (valid upper bound)
        Tq = np.empty(wg)
        for j in range(wg):
            own = tperm[qc[qi[j]] * leaf:(qc[qi[j]] + 1) * leaf]
            d = (q[j] ** 2).sum() + nc2[own] - 2 * np.einsum("tmk,k->tm", r4[own], q[j])
            Tq[j] = d.min()
        _, nd = oracle.nn_batch(rows, q.astype(np.float32))
        lb = (fq[qi] ** 2).sum(1)[:, None] + (fc ** 2).sum(1)[None] - 2 * fq[qi] @ fc.T  # [wg][T]
        surv = (lb[:, tperm] <= Tq[:, None] * (1 + 1e-6)).reshape(wg // wave, wave, T // tblk, tblk)
        need_wave = surv.any(3).any(1)  # [waves][tile blocks]
        frac.append(need_wave.mean())
        frac_wg.append(need_wave.any(0).mean())
        survd = (lb[:, tperm] <= nd[:, None] * (1 + 1e-6)).reshape(wg // wave, wave, T // tblk, tblk)
        frac_dstar.append(survd.any(3).any(1).mean())
        print("wg@%d clusters %s: need/wave %.3f need/WG %.3f (with d*: %.3f)  T_q/d* median %.2f" %
              (s, np.unique(qc[qi]).size, frac[-1], frac_wg[-1], frac_dstar[-1], np.median(Tq / nd)), flush=True)
    print("mean need per wave %.3f, per WG %.3f, ideal %.3f" % (np.mean(frac), np.mean(frac_wg), np.mean(frac_dstar)))



def bound_study(seed=7, nq=400, T=65536):
    """Tiles whose shortlist bound reaches the best true score (per query), for candidate bounds:
    (a) d0 + |d1| + |d2| + |d3|          (3 VALU adds per element)
    (b) d0 + sum_x |q_x|.|c_x|           (one accumulator: abs operands for blocks 1..3)
    (c) d0 + |d1| + sum_{x=2,3} |q_x|.|c_x|"""
    wl = synth.make_workload(seed, 1920, 1080, 1, T, n_palettes=128)
    used = synth.used_one_palette(wl.tile_pal, 128)
    rows, *_ = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    P = projections()
    Bs = []
    for x in range(4):
        w, V = np.linalg.eigh(P[x])
        Bs.append(V[:, w > 0.5])
    base = rows[0::4].astype(np.float64)
    cx = [base @ B for B in Bs]
    rng = np.random.default_rng(1)
    pick = rng.choice(wl.tiles_per_frame, nq, replace=False)
    q = oracle.psyv_batch(nq, rgb=wl.frame_rgb[0][pick], flags=2)
    qx = [q @ B for B in Bs]
    half_n = 0.5 * (base ** 2).sum(1)
    res = {k: [] for k in "abc"}
    ovf = {k: 0 for k in "abc"}
    nsb = {k: [] for k in "abc"}
    tt = np.arange(T)
    lst = ((tt // 32) * 4 // (T // 32)) * 2 + ((tt % 32) >> 2 & 1)  # list = split * 2 + lane half
    sub = tt // 4
    for i in range(nq):
        d = [cx[x] @ qx[x][i] for x in range(4)]
        sc = np.stack([d[0] + s1 * d[1] + s2 * d[2] + s1 * s2 * d[3] for s1 in (1, -1) for s2 in (1, -1)], 1)
        true = sc.max(1) - half_n
        best = true.max()
        ad = [np.abs(cx[x]) @ np.abs(qx[x][i]) for x in range(4)]
        bnd = {"a": d[0] + np.abs(d[1]) + np.abs(d[2]) + np.abs(d[3]) - half_n,
               "b": d[0] + ad[1] + ad[2] + ad[3] - half_n,
               "c": d[0] + np.abs(d[1]) + ad[2] + ad[3] - half_n}
        for k, b in bnd.items():
            res[k].append(int((b >= best).sum()))
            hit = np.unique(sub[b >= best])
            nsb[k].append(hit.size)
            if np.bincount(lst[hit * 4], minlength=8).max() >= 4:
                ovf[k] += 1
    for k in "abc":
        r = np.array(res[k])
        print("bound %s: tiles reaching the best score per query: mean %.1f median %.0f p90 %.0f max %d" %
              (k, r.mean(), np.median(r), np.quantile(r, 0.9), r.max()))
        print("   sub-blocks reaching best: mean %.1f; queries with a full list (>= 4 in one of 8 lists): %.2f%%"
              % (np.mean(nsb[k]), 100.0 * ovf[k] / nq))



def coarse_study(seed=7, T=65536, qblocks=6):
    """Shortlist list-test pass rates per (wave, 32-tile block) for the C3 workload: how often a wave-uniform
    test `any lane's bound > its list threshold` fires for (e) the exact per-tile bound d0 + sum |d_x| (the kernel's
    sub-block maxima), (s) a per-sub-block coarse bound max_t d0 + sum_x max_t |d_x| over the lane's 4 tiles, and
    (w) a per-lane coarse bound over the lane's 16 tiles of the block.  Lanes = 32 queries x 2 tile halves, lists of
    L = 4 sub-blocks by exact bound, blocks streamed in index order (nn_orbit_shortlist_pipe_kernel)."""
    wl = synth.make_workload(seed, 1920, 1080, 1, T, n_palettes=128)
    used = synth.used_one_palette(wl.tile_pal, 128)
    rows, *_ = oracle.build_ft_dataset(used, wl.tiles, wl.thm, wl.tvm, wl.palettes)
    P = projections()
    Bs = []
    for x in range(4):
        w, V = np.linalg.eigh(P[x])
        Bs.append(V[:, w > 0.5])
    base = rows[0::4].astype(np.float64)
    cx = [base @ B for B in Bs]
    half_n = 0.5 * (base ** 2).sum(1)
    nb = T // 32
    r = np.arange(16)
    rng = np.random.default_rng(5)
    tot = {k: [] for k in "esw"}
    for qb in rng.choice(wl.tiles_per_frame // 32, qblocks, replace=False):
        q = oracle.psyv_batch(32, rgb=wl.frame_rgb[0][qb * 32:(qb + 1) * 32], flags=2)
        d = [q @ B @ cx[x].T for x, B in enumerate(Bs)]  # [32][T]
        d[0] = d[0] - half_n[None]
        ex = d[0] + np.abs(d[1]) + np.abs(d[2]) + np.abs(d[3])
        lanes = []
        for h in (0, 1):
            tix = (np.arange(nb)[:, None] * 32 + ((r & 3) + 8 * (r >> 2) + 4 * h)[None]).reshape(-1)  # [nb*16]
            g = lambda a: a[:, tix].reshape(32, nb, 4, 4)  # noqa: E731  [q][blk][sub][tile]
            e4 = g(ex).max(3)
            s4 = g(d[0]).max(3) + sum(np.abs(g(d[x])).max(3) for x in (1, 2, 3))
            w1 = g(d[0]).max((2, 3)) + sum(np.abs(g(d[x])).max((2, 3)) for x in (1, 2, 3))
            lanes.append((e4, s4, w1))
        e4 = np.concatenate([l[0] for l in lanes])  # [64][nb][4]
        s4 = np.concatenate([l[1] for l in lanes])
        w1 = np.concatenate([l[2] for l in lanes])
        lst = np.full((64, 4), -np.inf)
        fire = {k: 0 for k in "esw"}
        for b in range(nb):
            th = lst.min(1)
            fire["e"] += bool((e4[:, b].max(1) > th).any())
            fire["s"] += bool((s4[:, b].max(1) > th).any())
            fire["w"] += bool((w1[:, b] > th).any())
            allv = np.concatenate([lst, e4[:, b]], 1)
            lst = -np.sort(-allv, 1)[:, :4]
        for k in "esw":
            tot[k].append(fire[k] / nb)
        print("qblock %d: fire rate exact %.4f  sub-block coarse %.4f  lane coarse %.4f" %
              (qb, fire["e"] / nb, fire["s"] / nb, fire["w"] / nb), flush=True)
    print("mean fire rate: exact %.4f  sub-block coarse %.4f  lane coarse %.4f" %
          tuple(np.mean(tot[k]) for k in "esw"))


if __name__ == "__main__":
    {"--ivf": ivf_study, "--blocks": block_study, "--bounds": bound_study, "--coarse": coarse_study}.get(sys.argv[-1], main)()

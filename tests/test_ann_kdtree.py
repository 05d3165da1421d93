"""CPU checks of the ANN 1.1.2 kd-tree restatement (oracle/ann_kdtree.c) and of the tie-order method the GPU
uses (tiler_amd/csrc/kdorder_dev.hpp, kdtree.hip), SURVEY.md 8(a) a8 / 8(c).

1. An independent numpy restatement of ANN's kd_tree constructor (annEnclRect, annMaxSpread, annMedianSplit,
   rkd_tree with kd_split) builds the same tree as the C oracle: split dims / values / cell bounds by split
   position, and the same leaf order.
2. The GPU's claim, checked on the oracle: the candidate annkSearch returns among equal distances is the one
   first in the depth-first order with q's near child first (decided at the two candidates' lowest common node),
   whenever every far-child box distance on its path is below the final k-th distance (the GPU's vouching
   check); k = 8 results are the 8 smallest by (distance, that order).
"""
import numpy as np
import pytest


def np_kdtree(data, bs=1):
    """numpy restatement of ANN's kd_tree(pa, n, dd, bs, ANN_KD_STD): pidx, and per split position m
    (cut_dim, cut_val, lo_bnd, hi_bnd)."""
    n, dd = data.shape
    pidx = list(range(n))
    cd = np.zeros(n, np.int32)
    cv = np.zeros(n, np.float32)
    lo_b = np.zeros(n, np.float32)
    hi_b = np.zeros(n, np.float32)
    lo = data.min(0).astype(np.float32) if n else np.zeros(dd, np.float32)
    hi = data.max(0).astype(np.float32) if n else np.zeros(dd, np.float32)

    def PA(i, d):
        return data[pidx[i], d]

    def median_split(s, cnt, d, n_lo):
        def sw(a, b):
            pidx[s + a], pidx[s + b] = pidx[s + b], pidx[s + a]
        C = lambda i: data[pidx[s + i], d]  # noqa: E731
        l, r = 0, cnt - 1
        while l < r:
            i = (r + l) // 2
            if C(i) > C(r):
                sw(i, r)
            sw(l, i)
            c = C(l)
            i, k = l, r
            while True:
                i += 1
                while C(i) < c:
                    i += 1
                k -= 1
                while C(k) > c:
                    k -= 1
                if i < k:
                    sw(i, k)
                else:
                    break
            sw(l, k)
            if k > n_lo:
                r = k - 1
            elif k < n_lo:
                l = k + 1
            else:
                break
        if n_lo > 0:
            c, k = C(0), 0
            for i in range(1, n_lo):
                if C(i) > c:
                    c, k = C(i), i
            sw(n_lo - 1, k)
        return np.float32((np.float32(C(n_lo - 1)) + np.float32(C(n_lo))) / np.float32(2))

    def build(s, cnt):
        if cnt <= bs:
            return
        pts = data[pidx[s:s + cnt]]
        spr = (pts.max(0) - pts.min(0)).astype(np.float32)
        d = int(np.argmax(spr)) if spr.max() > 0 else 0
        n_lo = cnt // 2
        v = median_split(s, cnt, d, n_lo)
        m = s + n_lo
        cd[m], cv[m], lo_b[m], hi_b[m] = d, v, lo[d], hi[d]
        sh = hi[d]
        hi[d] = v
        build(s, n_lo)
        hi[d] = sh
        sl = lo[d]
        lo[d] = v
        build(m, cnt - n_lo)
        lo[d] = sl

    build(0, n)
    return np.array(pidx, np.int32), cd, cv, lo_b, hi_b


def dfs_before(pos, cd, cv, n, bs, q, a, b):
    """kd_before (kdorder_dev.hpp) in Python"""
    pa, pb = pos[a], pos[b]
    sw = pa > pb
    if sw:
        pa, pb = pb, pa
    s, e = 0, n
    while e - s > bs:
        m = s + (e - s) // 2
        if pb < m:
            e = m
        elif pa >= m:
            s = m
        else:
            return bool((np.float32(q[cd[m]]) - np.float32(cv[m]) < 0) != sw)
    return not sw


def far_box(pos, cd, cv, lo_b, hi_b, n, bs, q, p, box_lo, box_hi):
    """kd_root_box + kd_path_far_box (kdorder_dev.hpp) in Python, fp32 op by op"""
    f = np.float32
    rb = f(0)
    for d in range(q.size):
        if q[d] < box_lo[d]:
            t = f(box_lo[d] - q[d])
            rb = f(rb + f(t * t))
        elif q[d] > box_hi[d]:
            t = f(q[d] - box_hi[d])
            rb = f(rb + f(t * t))
    box, worst = rb, f(-np.inf)
    s, e = 0, n
    while e - s > bs:
        m = s + (e - s) // 2
        qd = f(q[cd[m]])
        cut = f(qd - cv[m])
        lo_first, in_lo = bool(cut < 0), p < m
        if in_lo != lo_first:
            bd = f(lo_b[m] - qd) if lo_first else f(qd - hi_b[m])
            bd = max(bd, f(0))
            box = f(box + f(f(cut * cut) - f(bd * bd)))
            worst = max(worst, box)
        if in_lo:
            e = m
        else:
            s = m
    return worst


def exact_dists(data, q):
    f = np.float32
    d = np.zeros(data.shape[0], np.float32)
    for j in range(data.shape[1]):
        t = (q[j] - data[:, j]).astype(np.float32)
        d = (d + (t * t).astype(np.float32)).astype(np.float32)
    return d


def _datasets():
    rng = np.random.default_rng(5)
    base = rng.normal(0, 1, (40, 12)).astype(np.float32)
    dup = np.concatenate([base, base[::-1], base[:15]])             # every row 2-3 times
    ints = rng.integers(0, 4, (150, 10)).astype(np.float32)          # many equal coordinates and distances
    flat = np.repeat(rng.integers(0, 3, (30, 1)), 8, 1).astype(np.float32)
    flat = np.concatenate([flat, rng.integers(0, 3, (60, 8)).astype(np.float32)])
    return {"dup": dup, "ints": ints, "flat": flat}


@pytest.mark.parametrize("name", ["dup", "ints", "flat"])
@pytest.mark.parametrize("bs", [1, 3])
def test_oracle_tree_matches_numpy_restatement(oracle, name, bs):
    data = _datasets()[name]
    pidx, cd, cv, lo_b, hi_b = np_kdtree(data, bs)
    kd = oracle.KDTree(data, bs=bs)
    pos = kd.positions()
    assert np.array_equal(pos[pidx], np.arange(data.shape[0]))
    if bs == 1:
        ocd, ocv, olo, ohi = kd.splits()
        m = np.arange(1, data.shape[0])
        assert np.array_equal(ocd[m], cd[m])
        assert np.array_equal(ocv[m].view(np.uint32), cv[m].view(np.uint32))
        assert np.array_equal(olo[m].view(np.uint32), lo_b[m].view(np.uint32))
        assert np.array_equal(ohi[m].view(np.uint32), hi_b[m].view(np.uint32))
    kd.close()


@pytest.mark.parametrize("name", ["dup", "ints", "flat"])
@pytest.mark.parametrize("k", [1, 8])
def test_kd_result_is_first_in_dfs_order(oracle, name, k):
    """annkSearch == the k smallest by (distance, DFS order), for every query the path check vouches for."""
    data = _datasets()[name]
    rng = np.random.default_rng(11)
    n = data.shape[0]
    qs = np.concatenate([data[rng.integers(0, n, 40)], data[rng.integers(0, n, 40)] + rng.integers(-1, 2, (40, data.shape[1])),
                         rng.normal(0, 2, (40, data.shape[1]))]).astype(np.float32)
    kd = oracle.KDTree(data)
    ki, ke = kd.search_batch(qs, k=k)
    ki, ke = ki.reshape(len(qs), k), ke.reshape(len(qs), k)
    pos = kd.positions()
    cd, cv, lo_b, hi_b = kd.splits()
    kd.close()
    box_lo, box_hi = data.min(0), data.max(0)
    vouched = ties = 0
    import functools
    for qi, q in enumerate(qs):
        d = exact_dists(data, q)
        order = sorted(range(n), key=functools.cmp_to_key(
            lambda a, b: -1 if (d[a] < d[b] or (d[a] == d[b] and dfs_before(pos, cd, cv, n, 1, q, a, b))) else 1))
        want = np.array(order[:k], np.int32)
        Dk = d[want[-1]]
        ok = all((lambda fb: fb < Dk or (fb <= Dk and d[c] == Dk))(
            far_box(pos, cd, cv, lo_b, hi_b, n, 1, q, pos[c], box_lo, box_hi)) for c in want)
        ties += int(np.count_nonzero(d <= Dk) > k or np.unique(d[want]).size < k)
        if ok:
            vouched += 1
            assert np.array_equal(ki[qi], want), (qi, ki[qi], want)
            assert np.array_equal(ke[qi].view(np.uint32), d[want].view(np.uint32))
    assert vouched == len(qs)  # these exactly representable datasets never need the replay
    assert ties >= 3  # and they do exercise the tie rule


def py_pri_search(data, pidx, cd, cv, lo_b, hi_b, bs, q, eps):
    """annkPriSearch (ANN.dll 0x1800121a0, k = 1) in Python on the implicit tree of np_kdtree (node = leaf positions
    [s, e), split at m = s + (e - s) // 2), with ANNpr_queue's own binary heap (its tie behaviour is part of the
    order), fp32 op by op -- independent of oracle/ann_kdtree.c's explicit-node restatement."""
    f = np.float32
    n, dd = data.shape
    max_err = f(f(eps) + f(1))
    max_err = f(max_err * max_err)
    lo, hi = data.min(0), data.max(0)
    box = f(0)
    for d in range(dd):
        if q[d] < lo[d]:
            t = f(lo[d] - q[d])
            box = f(box + f(t * t))
        elif q[d] > hi[d]:
            t = f(q[d] - hi[d])
            box = f(box + f(t * t))
    pq = [None]  # 1-based

    def insert(kv, node):
        pq.append(None)
        r = len(pq) - 1
        while r > 1:
            p = r // 2
            if pq[p][0] <= kv:
                break
            pq[r] = pq[p]
            r = p
        pq[r] = (kv, node)

    def extr_min():
        top = pq[1]
        kn = pq[-1][0]
        last = pq[-1]
        nn = len(pq) - 2
        p, r = 1, 2
        while r <= nn:
            if r < nn and pq[r][0] > pq[r + 1][0]:
                r += 1
            if kn <= pq[r][0]:
                break
            pq[p] = pq[r]
            p, r = r, 2 * r
        pq[p] = last
        pq.pop()
        return top

    best, best_i = None, -1
    insert(box, (0, n))
    while len(pq) > 1:
        kv, (s, e) = extr_min()
        if f(kv * max_err) >= (best if best is not None else f(np.finfo(np.float32).max)):
            break
        while e - s > bs:
            m = s + (e - s) // 2
            qd = f(q[cd[m]])
            cut = f(qd - cv[m])
            if cut < 0:
                bd = f(lo_b[m] - qd)
                bd = bd if bd > 0 else f(0)
                insert(f(f(f(cut * cut) - f(bd * bd)) + kv), (m, e))
                e = m
            else:
                bd = f(qd - hi_b[m])
                bd = bd if bd > 0 else f(0)
                insert(f(f(f(cut * cut) - f(bd * bd)) + kv), (s, m))
                s = m
        min_dist = best if best is not None else f(np.finfo(np.float32).max)
        for lp in range(s, e):
            j = int(pidx[lp])
            dist = f(0)
            done = True
            for d in range(dd):
                t = f(q[d] - data[j, d])
                dist = f(dist + f(t * t))
                if dist > min_dist:
                    done = False
                    break
            if done:
                if best is None or best > dist:
                    best, best_i = dist, j
                min_dist = best
    return best_i, (best if best is not None else f(np.finfo(np.float32).max))


@pytest.mark.parametrize("name", ["dup", "ints", "flat"])
@pytest.mark.parametrize("bs", [1, 3])
@pytest.mark.parametrize("eps", [0.0, 0.5])
def test_oracle_pri_search_matches_python_restatement(oracle, name, bs, eps):
    """or_kdtree_pri_search_batch (ann_kdtree_pri_search's checker) == the Python restatement above, index and
    distance bits; with eps = 0 the distance is the exact minimum (only the choice among ties is the search's)."""
    data = _datasets()[name]
    rng = np.random.default_rng(17)
    n = data.shape[0]
    qs = np.concatenate([data[rng.integers(0, n, 30)], data[rng.integers(0, n, 30)] + rng.integers(-1, 2, (30, data.shape[1])),
                         rng.normal(0, 2, (30, data.shape[1]))]).astype(np.float32)
    pidx, cd, cv, lo_b, hi_b = np_kdtree(data, bs)
    kd = oracle.KDTree(data, bs=bs)
    oi, oe = kd.pri_search_batch(qs, eps)
    si, se = kd.search_batch(qs)
    kd.close()
    differ = 0
    for qi, q in enumerate(qs):
        pi_, pe_ = py_pri_search(data, pidx, cd, cv, lo_b, hi_b, bs, q, eps)
        assert oi[qi] == pi_ and np.float32(oe[qi]).view(np.uint32) == np.float32(pe_).view(np.uint32), qi
        if eps == 0.0:
            assert oe[qi] == exact_dists(data, q).min()
            differ += int(oi[qi] != si[qi])
    if eps == 0.0 and name == "ints":
        assert differ > 0  # the priority search's tie order is its own (ann_kdtree_search would answer otherwise)


@pytest.mark.parametrize("name", ["dup", "ints", "flat"])
@pytest.mark.parametrize("bs", [1, 3])
def test_pri_search_entry_key_rule(oracle, name, bs):
    """The GPU's fast priority-search answer (kdtree.hip kd_pri_resolve_kernel), checked on the oracle: with D the
    exact minimum and S the points at D, annkPriSearch returns the point of S with the smallest leaf entry key
    (the box value after the last far step on its path) below D, bucket order inside one leaf -- whenever that
    minimum is below D and held by a single leaf (otherwise the GPU replays)."""
    data = _datasets()[name]
    rng = np.random.default_rng(23)
    n = data.shape[0]
    qs = np.concatenate([data[rng.integers(0, n, 40)], data[rng.integers(0, n, 40)] + rng.integers(-1, 2, (40, data.shape[1])),
                         rng.normal(0, 2, (40, data.shape[1]))]).astype(np.float32)
    kd = oracle.KDTree(data, bs=bs)
    oi, oe = kd.pri_search_batch(qs)
    pos = kd.positions()
    kd.close()
    pidx, cd, cv, lo_b, hi_b = np_kdtree(data, bs)
    box_lo, box_hi = data.min(0), data.max(0)

    def leaf_start(p):
        s, e = 0, n
        while e - s > bs:
            m = s + (e - s) // 2
            s, e = (s, m) if p < m else (m, e)
        return s

    decided = 0
    for qi, q in enumerate(qs):
        d = exact_dists(data, q)
        dm = d.min()
        S = np.nonzero(d == dm)[0]
        f = np.float32
        rbv = f(0)  # annBoxDistance: the root's own entry key
        for dd in range(q.size):
            if q[dd] < box_lo[dd]:
                t = f(box_lo[dd] - q[dd])
                rbv = f(rbv + f(t * t))
            elif q[dd] > box_hi[dd]:
                t = f(q[dd] - box_hi[dd])
                rbv = f(rbv + f(t * t))
        eks = []
        for p in S:
            w = far_box(pos, cd, cv, lo_b, hi_b, n, bs, q, int(pos[p]), box_lo, box_hi)
            eks.append(rbv if w == f(-np.inf) else w)  # no far step on the path: the root's chain
        eks = np.array(eks, np.float32)
        ekm = eks.min()
        cand = S[eks == ekm]
        leaves = {leaf_start(int(pos[p])) for p in cand}
        if not (ekm < dm and len(leaves) == 1):
            continue
        decided += 1
        want = cand[np.argmin(pos[cand])]
        assert oi[qi] == want and oe[qi] == dm, qi
    assert decided >= len(qs) // 2

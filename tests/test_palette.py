"""CPU tests of palette generation: the oracle's DLv3 restatement (oracle/palette.c) against
an independent pure-Python restatement of dlquant/quantizer.c:437-663 on small colour sets, RGBToHSV / MulDiv
known answers, the CompareCMULHS and FinishQuantizePalette orders, and the product's host-side order function.
quantizer.c itself is not buildable here (MSVC-only declarations, mtPaint progress callbacks, conflicting
calc_err declarations), so DLv3 parity is unpinned against the reference binary."""
import numpy as np
import pytest

F32 = np.float32


def _py_dl3quant(px, quant_to=16, bpc=7):
    """quantizer.c:437-663 line by line in Python ints + numpy float32 (32-bit wrapping sums)."""
    M = 0xFFFFFFFF
    mbpc = (1 << bpc) - 1
    table = {}
    for r, g, b in px.tolist():
        idx = ((b * mbpc) // 255) | (((g * mbpc) // 255) << bpc) | (((r * mbpc) // 255) << (2 * bpc))
        e = table.setdefault(idx, [0, 0, 0, 0])
        e[0] = (e[0] + r) & M
        e[1] = (e[1] + g) & M
        e[2] = (e[2] + b) & M
        e[3] = (e[3] + 1) & M
    T = []

    def setrgb(e):
        v = e[3]
        v2 = v >> 1
        e[4:7] = [((e[0] + v2) & M) // v & 255, ((e[1] + v2) & M) // v & 255, ((e[2] + v2) & M) // v & 255]

    for k in sorted(table):
        e = table[k] + [0, 0, 0, F32(0), 0]
        setrgb(e)
        T.append(e)

    def calc_err(a, b):
        A, B = T[a], T[b]
        P1, P2 = A[3], B[3]
        P3 = (P1 + P2) & M
        R3 = ((A[0] + B[0] + (P3 >> 1)) & M) // P3
        G3 = ((A[1] + B[1] + (P3 >> 1)) & M) // P3
        B3 = ((A[2] + B[2] + (P3 >> 1)) & M) // P3
        d1 = F32(F32((R3 - A[4]) ** 2) + F32((G3 - A[5]) ** 2)) + F32((B3 - A[6]) ** 2)
        d1 = F32(np.sqrt(F32(d1)) * F32(P1))
        d2 = F32(F32((B[4] - R3) ** 2) + F32((B[5] - G3) ** 2)) + F32((B[6] - B3) ** 2)
        d2 = F32(np.sqrt(F32(d2)) * F32(P2))
        return F32(d1 + d2)

    tot = [len(T)]
    INF = F32(np.inf)

    def recount_next(i):
        err, c2 = INF, 0
        for j in range(i + 1, tot[0]):
            cur = calc_err(i, j)
            if cur < err:
                err, c2 = cur, j
        T[i][7], T[i][8] = err, c2

    def recount_dist(c1):
        recount_next(c1)
        for i in range(c1):
            if T[i][8] == c1:
                recount_next(i)
            else:
                cur = calc_err(i, c1)
                if cur < T[i][7]:
                    T[i][7], T[i][8] = cur, c1

    for i in range(tot[0] - 1):
        recount_next(i)
    if tot[0]:
        T[tot[0] - 1][7], T[tot[0] - 1][8] = INF, tot[0]
    c1 = 0
    while tot[0] > quant_to:
        err = INF
        for i in range(tot[0]):
            if T[i][7] < err:
                err, c1 = T[i][7], i
        c2 = T[c1][8]
        for k in range(4):
            T[c2][k] = (T[c2][k] + T[c1][k]) & M
        setrgb(T[c2])
        tot[0] -= 1
        T[c1] = list(T[tot[0]])
        T[tot[0] - 1][7], T[tot[0] - 1][8] = INF, tot[0]
        for i in range(c1):
            if T[i][8] == tot[0]:
                T[i][8] = c1
        for i in range(c1 + 1, tot[0]):
            if T[i][8] == tot[0]:
                recount_next(i)
        recount_dist(c1)
        if c2 != tot[0]:
            recount_dist(c2)
    return np.array([T[i][4] | (T[i][5] << 8) | (T[i][6] << 16) if i < tot[0] else 0 for i in range(quant_to)],
                    np.int32)


def _pixels(rng, n, kind):
    if kind == "noise":
        return rng.integers(0, 256, (n, 3)).astype(np.uint8)
    if kind == "few":  # fewer cells than quant_to
        base = rng.integers(0, 256, (5, 3))
        return base[rng.integers(0, 5, n)].astype(np.uint8)
    base = rng.integers(0, 256, (12, 3))  # clustered: ties in calc_err are common
    return np.clip(base[rng.integers(0, 12, n)] + rng.integers(-6, 7, (n, 3)), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("kind,n,bpc", [("noise", 120, 7), ("clustered", 400, 7), ("few", 50, 7), ("noise", 150, 5),
                                        ("clustered", 300, 4)])
def test_oracle_dl3quant_matches_python_restatement(oracle, kind, n, bpc):
    px = _pixels(np.random.default_rng(n + bpc), n, kind)
    got, hist = oracle.dl3quant(px, 16, bpc)
    assert np.array_equal(got, _py_dl3quant(px, 16, bpc))


def test_oracle_dl3quant_empty_and_single(oracle):
    got, hist = oracle.dl3quant(np.zeros((0, 3), np.uint8))
    assert hist == 0 and not got.any()
    got, hist = oracle.dl3quant(np.array([[10, 20, 30]] * 7, np.uint8))
    assert hist == 1 and got[0] == (10 | 20 << 8 | 30 << 16) and not got[1:].any()


def _muldiv(a, b, c):
    """Windows MulDiv: the operands' signs pick +-c/2, then C division (truncation toward zero)."""
    if c < 0:
        a, c = -a, -c
    r = a * b + (c // 2 if (a < 0) == (b < 0) or (a >= 0 and b >= 0) else -(c // 2))
    return r // c if r >= 0 else -((-r) // c)


def _py_hsv(col):
    rr, gg, bb = col & 255, (col >> 8) & 255, (col >> 16) & 255
    mx, mn = max(rr, gg, bb), min(rr, gg, bb)
    hh = ss = 0
    if mx != mn:
        d = mx - mn
        ss = _muldiv(d, 255, mx)
        if rr == mx:
            hh = _muldiv(42, gg - bb, d)
        elif gg == mx:
            hh = _muldiv(42, bb - rr, d) + 84
        else:
            hh = _muldiv(42, rr - gg, d) + 168
        hh = int(np.fmod(hh, 252))
    return hh & 255, ss & 255, mx


def test_oracle_hsv(oracle):
    assert oracle.rgb_to_hsv(0x0000FF) == (0, 255, 255)  # red
    assert oracle.rgb_to_hsv(0x00FF00) == (84, 255, 255)  # green
    assert oracle.rgb_to_hsv(0xFF0000) == (168, 255, 255)  # blue
    assert oracle.rgb_to_hsv(0xFF00FF) == (214, 255, 255)  # magenta: -42 mod 252 -> byte
    assert oracle.rgb_to_hsv(0x808080) == (0, 0, 128)
    rng = np.random.default_rng(3)
    for col in rng.integers(0, 1 << 24, 3000).tolist():
        assert oracle.rgb_to_hsv(col) == _py_hsv(col), hex(col)


def test_sort_cmulhs_orders_by_luma_val_sat_hue(oracle):
    rng = np.random.default_rng(4)
    cols = rng.integers(0, 1 << 24, 16).astype(np.int32)
    cols[3] = cols[9]  # duplicates: equal keys
    out = oracle.sort_cmulhs(cols)
    assert sorted(out.tolist()) == sorted(cols.tolist())

    def key(c):
        h, s, v = oracle.rgb_to_hsv(int(c))
        return ((c & 255) * 2126 + ((c >> 8) & 255) * 7152 + ((c >> 16) & 255) * 722) // 10000, v, s, h
    keys = [key(int(c)) for c in out]
    assert keys == sorted(keys)


@pytest.mark.parametrize("uc", [[5, 9, 9, 1, 5], [0] * 8, list(range(16)), [3, 3, 3, 7, 7, 1, 0, 7, 2]])
def test_finish_quantize_order_product_matches_oracle(oracle, uc):
    """FinishQuantizePalette's order (host code in libANN.so, no GPU needed) equals the oracle's kmodes.pas
    QuickSort restatement; use counts come out descending."""
    from tiler_amd.palette import finish_quantize_order
    lut = finish_quantize_order(uc)
    assert np.array_equal(lut, oracle.finish_quantize_order(uc))
    order = np.argsort(lut)
    assert sorted(lut.tolist()) == list(range(len(uc)))
    assert all(uc[order[i]] >= uc[order[i + 1]] for i in range(len(uc) - 1))


def _lab_float(r, g, b):
    """RGBToLAB (main.pas:2711-2747) with Python's libm, gamma -1: the oracle's fdlibm path agrees to ~1 ulp."""
    def lin(v):
        v = v / 255.0
        return ((v + 0.055) / 1.055) ** 2.4 if v > 0.04045 else v / 12.92
    r, g, b = lin(r), lin(g), lin(b)
    x = (r * 0.49 + g * 0.31 + b * 0.2) / 0.17697 / (96.6797 / 100)
    y = (r * 0.17697 + g * 0.8124 + b * 0.01063) / 0.17697
    z = (g * 0.01 + b * 0.99) / 0.17697 / (82.5188 / 100)
    f = [t ** (1 / 3) if t > 0.008856 else 7.787 * t + 16 / 116 for t in (x, y, z)]
    return 116 * f[1] - 16, 500 * (f[0] - f[1]), 200 * (f[1] - f[2])


def test_oracle_lab_descriptor(oracle):
    """A flat tile's LAB + Haar descriptor holds 8 x the LAB value in its DC terms and zeros elsewhere."""
    for r, g, b in [(255, 255, 255), (0, 0, 0), (200, 30, 90), (5, 8, 3)]:
        tile = np.full((1, 64), r | g << 8 | b << 16, np.int32)
        d = oracle.psyv_lab_batch(tile)[0]
        want = _lab_float(r, g, b)
        for c in range(3):
            assert abs(d[c * 64] - 8 * want[c]) < 1e-9 * max(1.0, abs(want[c])) * 8
            assert np.all(np.abs(d[c * 64 + 1:(c + 1) * 64]) < 1e-12)


def test_oracle_kmeans_separated_clusters(oracle):
    rng = np.random.default_rng(8)
    centers = rng.normal(0, 50, (6, 192))
    lab = rng.integers(0, 6, 1200)
    X = centers[lab] + rng.normal(0, 1, (1200, 192))
    labels, cent, it = oracle.kmeans(X, 6)
    assert it >= 2
    # every found cluster is one true cluster (k-means++ on well separated data)
    for c in range(6):
        assert np.unique(lab[labels == c]).size == 1
    for c in range(6):
        m = labels == c
        assert np.allclose(cent[c], X[m].mean(0), rtol=0, atol=1e-9)


# The GPU's pass-2 order (palette.hip dl3_reduce_kernel): the moved-entry fix-ups, recount_dist(c1)'s loop and
# every recount of the merge run as ONE pass whose lanes may go in any order, then recount_dist(c2); the minimum
# error comes from chunk minima (equal to the plain first minimum).  This model runs the lanes of each parallel
# phase in a random order and must reproduce the sequential restatement exactly.
def _py_dl3quant_gpu_order(px, quant_to=16, bpc=7, order_seed=0):
    import random
    rnd = random.Random(order_seed)
    M = 0xFFFFFFFF
    mbpc = (1 << bpc) - 1
    table = {}
    for r, g, b in px.tolist():
        idx = ((b * mbpc) // 255) | (((g * mbpc) // 255) << bpc) | (((r * mbpc) // 255) << (2 * bpc))
        e = table.setdefault(idx, [0, 0, 0, 0]); e[0]=(e[0]+r)&M; e[1]=(e[1]+g)&M; e[2]=(e[2]+b)&M; e[3]=(e[3]+1)&M
    T = []
    def setrgb(e):
        v = e[3]; v2 = v >> 1
        e[4:7] = [((e[0]+v2)&M)//v & 255, ((e[1]+v2)&M)//v & 255, ((e[2]+v2)&M)//v & 255]
    for k in sorted(table):
        e = table[k] + [0,0,0, F32(0), 0]; setrgb(e); T.append(e)
    def calc_err(a, b):
        A, B = T[a], T[b]; P1, P2 = A[3], B[3]; P3 = (P1+P2)&M
        R3 = ((A[0]+B[0]+(P3>>1))&M)//P3; G3 = ((A[1]+B[1]+(P3>>1))&M)//P3; B3 = ((A[2]+B[2]+(P3>>1))&M)//P3
        d1 = F32(F32(F32((R3-A[4])**2) + F32((G3-A[5])**2)) + F32((B3-A[6])**2)); d1 = F32(np.sqrt(d1) * F32(P1))
        d2 = F32(F32(F32((B[4]-R3)**2) + F32((B[5]-G3)**2)) + F32((B[6]-B3)**2)); d2 = F32(np.sqrt(d2) * F32(P2))
        return F32(d1 + d2)
    INF = F32(np.inf)
    tot = len(T)
    def recount_next(i):
        err, c2 = INF, 0
        for j in range(i+1, tot):
            cur = calc_err(i, j)
            if cur < err: err, c2 = cur, j
        T[i][7], T[i][8] = err, c2
    for i in range(tot-1): recount_next(i)
    if tot: T[tot-1][7], T[tot-1][8] = INF, tot
    c1 = 0
    while tot > quant_to:
        # argmin via chunk minima == plain first minimum
        err = INF
        for i in range(tot):
            if T[i][7] < err: err, c1 = T[i][7], i
        c2 = T[c1][8]
        for k in range(4): T[c2][k] = (T[c2][k] + T[c1][k]) & M
        setrgb(T[c2]); tot -= 1
        T[c1] = list(T[tot]); T[tot-1][7], T[tot-1][8] = INF, tot
        # fused pass B, lanes in random order
        lst = []
        idxs = [i for i in range(tot) if i != c1]; rnd.shuffle(idxs)
        for i in idxs:
            ci = T[i][8]
            if i > c1:
                if ci == tot: lst.append(i)
                continue
            if ci == tot: ci = c1; T[i][8] = c1
            if ci == c1: lst.append(i)
            else:
                cur = calc_err(i, c1)
                if cur < T[i][7]: T[i][7], T[i][8] = cur, c1
        lst.append(c1); rnd.shuffle(lst)
        for i in lst: recount_next(i)
        if c2 != tot:
            recount_next(c2)
            l2 = []
            idxs = list(range(c2)); rnd.shuffle(idxs)
            for i in idxs:
                if T[i][8] == c2: l2.append(i)
                else:
                    cur = calc_err(i, c2)
                    if cur < T[i][7]: T[i][7], T[i][8] = cur, c2
            rnd.shuffle(l2)
            for i in l2: recount_next(i)
    return np.array([T[i][4] | (T[i][5] << 8) | (T[i][6] << 16) if i < tot else 0 for i in range(quant_to)], np.int32)



@pytest.mark.parametrize("seed", range(9))
def test_dl3_gpu_phase_order_equals_sequential(seed):
    kind = ["noise", "clustered", "few"][seed % 3]
    px = _pixels(np.random.default_rng(100 + seed), [150, 300, 60][seed % 3], kind)
    assert np.array_equal(_py_dl3quant_gpu_order(px, 16, 7, seed), _py_dl3quant(px, 16, 7))

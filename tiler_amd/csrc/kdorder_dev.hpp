// kdorder_dev.hpp -- device side of the ANN tie order (kdtree.hpp): which of two equal-distance candidates
// annkSearch finds first, and ANN's box-distance pruning replayed along one candidate's path.
#pragma once
#include <float.h>
#include <hip/hip_runtime.h>

#include "kdtree.hpp"

#pragma clang fp contract(off)

namespace tiler {

// True iff candidate a is visited before candidate b by ANN's depth-first search for query q (near child
// first: LO when q[cd] - cv < 0, ANNkd_split::ann_search).  Order of the visit over ALL leaves: at the two
// candidates' lowest common node, the one in q's near child comes first; inside one bucket, position order
// (ANNkd_leaf::ann_search scans bkt[] in order).  op == nullptr (no tree): the lower index.  Invalid ids
// (< 0 or >= n, e.g. the 0x7fffffff "none" sentinel) come after every valid one.  The view is read through
// a pointer, and only here: search kernels carry 8 bytes of argument for it and touch it on exact ties only.
static __device__ __attribute__((noinline)) bool kd_before_tree(const KdOrder *__restrict__ op, const float *__restrict__ q,
                                                         int a, int b) {
    const KdOrder &o = *op;
    if ((unsigned)a >= (unsigned)o.n || (unsigned)b >= (unsigned)o.n) return (unsigned)a < (unsigned)b;
    int pa = o.pos[a], pb = o.pos[b];
    const bool sw = pa > pb;
    if (sw) {
        const int t = pa;
        pa = pb;
        pb = t;
    }
    int s = 0, e = o.n;
    while (e - s > o.bs) {
        const int m = s + ((e - s) >> 1);
        if (pb < m) {
            e = m;
        } else if (pa >= m) {
            s = m;
        } else {
            const float cut_diff = q[o.cd[m]] - o.cv[m];
            return (cut_diff < 0.0f) != sw;
        }
    }
    return !sw;
}

__device__ __forceinline__ bool kd_before(const KdOrder *op, const float *__restrict__ q, int a, int b) {
    return op ? kd_before_tree(op, q, a, b) : (unsigned)a < (unsigned)b;
}

// kd_before as a 32-bit key: the root-to-leaf path of candidate c's leaf, one bit per internal node (0 = q's near
// child), then the position inside the bucket, left-aligned.  The paths of two leaves first differ at their lowest
// common node, so unsigned comparison of the keys is exactly kd_before (bs = 1: ceil(log2 n) <= 31 bits; in general
// the path and the bucket offset need <= ceil(log2 n) + 1 <= 32 bits for n < 2^31).  op == nullptr: the index.
// Tier 2 (orbit.hip) packs (distance bits, this key) into one u64 and takes an atomic minimum.
static __device__ __attribute__((noinline, unused)) unsigned kd_rank(const KdOrder *__restrict__ op, const float *__restrict__ q,
                                                             int c) {
    if (!op) return (unsigned)c;
    const KdOrder &o = *op;
    const int p = o.pos[c];
    unsigned bits = 0;
    int nb = 0, s = 0, e = o.n;
    while (e - s > o.bs) {
        const int m = s + ((e - s) >> 1);
        const bool lo_first = (q[o.cd[m]] - o.cv[m]) < 0.0f, in_lo = p < m;
        bits = (bits << 1) | (in_lo == lo_first ? 0u : 1u);
        nb++;
        if (in_lo)
            e = m;
        else
            s = m;
    }
    const int bb = o.bs > 1 ? 32 - __builtin_clz((unsigned)(o.bs - 1)) : 0;  // ceil(log2 bs)
    bits = (bb ? (bits << bb) : bits) | (unsigned)(p - s);
    nb += bb;
    return nb == 0 ? 0u : bits << (32 - nb);
}

// the candidate whose kd_rank is r (same walk, following the key's bits)
static __device__ __attribute__((noinline, unused)) int kd_unrank(const KdOrder *__restrict__ op, const float *__restrict__ q,
                                                          unsigned r) {
    if (!op) return (int)r;
    const KdOrder &o = *op;
    int s = 0, e = o.n, used = 0;
    while (e - s > o.bs) {
        const int m = s + ((e - s) >> 1);
        const bool lo_first = (q[o.cd[m]] - o.cv[m]) < 0.0f;
        const bool far = (r >> (31 - used)) & 1u;
        used++;
        if (lo_first != far)  // near child LO and bit 0, or far child LO and bit 1
            e = m;
        else
            s = m;
    }
    const int bb = o.bs > 1 ? 32 - __builtin_clz((unsigned)(o.bs - 1)) : 0;
    const int off = bb ? (int)((r << used) >> (32 - bb)) : 0;
    return o.pidx[s + off];
}

// (dist, kd order) lexicographic "less"
__device__ __forceinline__ bool kd_less(const KdOrder *op, const float *__restrict__ q, float da, int a, float db,
                                        int b) {
    return da < db || (da == db && kd_before(op, q, a, b));
}

// Insert (x, xi) into a lane's K-list (bd, bi) sorted by (distance, ANN order), as the shifting insertion
//     p = n;  while (p > 0 && kd_less(x, list[p-1])) { list[p] = list[p-1]; p--; }  list[p] = x;
// does (n = the slot that receives the last entry: K - 1 for a full list, the count while it fills; the caller has
// already checked that x enters the list) -- in two phases.  First the position: the test of every slot below n,
// the tie walk only on an equal distance, no list register written.  Then the move: straight-line selects on the
// known position, no call and no branch.  The shifting loop itself is miscompiled by this toolchain (ROCm 7.2, gfx950)
// when its tie test is more than one block (the kd_before_tree call, inlined or not): the shifted copy of the list is
// formed ahead of the divergent tie test, and the join's phi copies -- the unshifted list, for the lanes whose test
// fails -- are placed in the structurizer's flow block, which the lanes whose tie test succeeds execute too, into the
// same registers; such a lane then keeps an unshifted slot, so one entry is lost and its neighbour listed twice.  The
// optimised LLVM IR is correct, the ISA is not (DESIGN §4 "A k = 8 correctness fix", tools/merge_tie_repro.hip,
// profiles/r06/tie_repro.txt: 53-57 of 64 lanes corrupted; 0 with the tie test a single compare, 0 in this form).
template <int K>
__device__ __forceinline__ void kd_list_insert(const KdOrder *op, const float *__restrict__ q, float (&bd)[K],
                                               int (&bi)[K], float x, int xi, int n = K - 1) {
    bool f[K];
#pragma unroll
    for (int i = 0; i < K - 1; i++) f[i] = i < n && kd_less(op, q, x, xi, bd[i], bi[i]);
    int p = n;  // the loop's stop: the lowest slot of the run of passed tests that ends at slot n - 1
#pragma unroll
    for (int i = K - 2; i >= 0; i--)
        if (f[i] && p == i + 1) p = i;
#pragma unroll
    for (int i = K - 1; i > 0; i--) {
        const bool sh = i > p && i <= n;
        bd[i] = sh ? bd[i - 1] : (i == p ? x : bd[i]);
        bi[i] = sh ? bi[i - 1] : (i == p ? xi : bi[i]);
    }
    bd[0] = p == 0 ? x : bd[0];
    bi[0] = p == 0 ? xi : bi[0];
}

// (dist, kd order) minimum over lanes xor-reachable below `width` (64: the wave, 32: a half-wave, 4: a quad)
template <int WIDTH>
__device__ __forceinline__ void kd_argmin(const KdOrder *o, const float *__restrict__ q, float &v, int &i) {
#pragma unroll
    for (int off = WIDTH / 2; off > 0; off >>= 1) {
        const float ov = __shfl_xor(v, off, 64);
        const int oi = __shfl_xor(i, off, 64);
        if (kd_less(o, q, ov, oi, v, i)) {
            v = ov;
            i = oi;
        }
    }
}

// annBoxDistance(q, bnd_box_lo, bnd_box_hi, dim): fp32, dimension order, every op rounded
__device__ __forceinline__ float kd_root_box(const KdOrder &o, const float *__restrict__ q) {
    float dist = 0.0f;
    for (int d = 0; d < o.dd; d++) {
        const float v = q[d], lo = o.box_lo[d], hi = o.box_hi[d];
        if (v < lo) {
            const float t = lo - v;
            dist = dist + t * t;
        } else if (v > hi) {
            const float t = v - hi;
            dist = dist + t * t;
        }
    }
    return dist;
}

// The same value by a whole wave (every lane returns it): lanes load and square 64 dimensions at a time, the outside
// terms are then added in dimension order from registers -- the sequential sum without a memory round trip per term
__device__ __forceinline__ float kd_root_box_wave(const KdOrder &o, const float *__restrict__ q, int lane) {
    float rb = 0.0f;
    for (int d00 = 0; d00 < o.dd; d00 += 256) {  // 4 pieces of 64 dimensions: their loads in flight together
        float t[4];
        bool outside[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int d = d00 + 64 * u + lane;
            t[u] = 0.0f;
            outside[u] = false;
            if (d < o.dd) {
                const float v = q[d], lo = o.box_lo[d], hi = o.box_hi[d];
                if (v < lo) {
                    t[u] = lo - v;
                    outside[u] = true;
                } else if (v > hi) {
                    t[u] = v - hi;
                    outside[u] = true;
                }
                t[u] = t[u] * t[u];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            unsigned long long m = __ballot(outside[u]);
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1;
                rb = rb + __shfl(t[u], src, 64);
            }
        }
    }
    return rb;
}

// kd_path_far_box by a half-wave (h = lane >> 5; p uniform over the half): lane l of the half loads path level l, all
// levels in flight together, then every lane of the half adds the far-child terms in path order from shuffles --
// the same sequential fp32 sum.  Path depth <= 32 (as kd_quad_path_ok).
__device__ __forceinline__ float kd_half_path_far_box(const KdOrder &o, const float *__restrict__ q, int p,
                                                      float root_box, int lane) {
    const int l = lane & 31, base = lane & 32;
    int S = 0, E = o.n, m = -1;
    bool in_lo = false;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        if (E - S > o.bs) {
            const int mm = S + ((E - S) >> 1);
            const bool lo = p < mm;
            if (i == l) {
                m = mm;
                in_lo = lo;
            }
            if (lo)
                E = mm;
            else
                S = mm;
        }
    }
    float term = 0.0f;
    bool far = false;
    if (m >= 0) {
        const float qd = q[o.cd[m]];
        const float cut_diff = qd - o.cv[m];
        const bool lo_first = cut_diff < 0.0f;
        if (in_lo != lo_first) {
            float box_diff = lo_first ? o.lo[m] - qd : qd - o.hi[m];
            if (box_diff < 0.0f) box_diff = 0.0f;
            term = cut_diff * cut_diff - box_diff * box_diff;
            far = true;
        }
    }
    const unsigned fm = (unsigned)(__ballot(far) >> base);
    float box = root_box, worst = -INFINITY;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const float t = __shfl(term, base + i, 64);
        if ((fm >> i) & 1) {
            box = box + t;
            worst = fmaxf(worst, box);
        }
    }
    return worst;
}

// The largest box distance ANN computes for a far child on the root-to-leaf path of leaf position p
// (ANNkd_split::ann_search: box_dist + (cut_diff^2 - box_diff^2), fp32).  The leaf is visited iff every one of
// these is < the k-th key current at that check; -inf when p lies only in near children.
__device__ __forceinline__ float kd_path_far_box(const KdOrder &o, const float *__restrict__ q, int p, float root_box) {
    float box = root_box, worst = -INFINITY;
    int s = 0, e = o.n;
    while (e - s > o.bs) {
        const int m = s + ((e - s) >> 1);
        const float qd = q[o.cd[m]];
        const float cut_diff = qd - o.cv[m];
        const bool lo_first = cut_diff < 0.0f, in_lo = p < m;
        if (in_lo != lo_first) {
            float box_diff = lo_first ? o.lo[m] - qd : qd - o.hi[m];
            if (box_diff < 0.0f) box_diff = 0.0f;
            box = box + (cut_diff * cut_diff - box_diff * box_diff);
            worst = fmaxf(worst, box);
        }
        if (in_lo)
            e = m;
        else
            s = m;
    }
    return worst;
}

// The same check for ONE candidate by the 4 lanes of a quad (lane s = 0..3 of the quad, quad-uniform p): lane s
// loads the path levels l = s mod 4 (the q row is cache-hot in the pair pass that calls this), lane 0 of the quad
// adds the far-child terms in path order exactly as ANN does.  Returns, on every lane of the quad, whether every
// far-child box distance on p's path is <= D (k = 1: the winner's own distance; see kd_verify_kernel).
__device__ __forceinline__ bool kd_quad_path_ok(const KdOrder *__restrict__ op, const float *__restrict__ q, int p,
                                                float root_box, float D, int s) {
    const KdOrder &o = *op;
    float term[8];
    unsigned farm = 0;  // bit l: level l is a far step
#pragma unroll
    for (int i = 0; i < 8; i++) term[i] = 0.0f;
    int S = 0, E = o.n;
#pragma unroll
    for (int l = 0; l < 32; l++) {
        if (E - S > o.bs) {
            const int m = S + ((E - S) >> 1);
            const bool in_lo = p < m;
            if ((l & 3) == s) {
                const float qd = q[o.cd[m]];
                const float cut_diff = qd - o.cv[m];
                const bool lo_first = cut_diff < 0.0f;
                if (in_lo != lo_first) {
                    float box_diff = lo_first ? o.lo[m] - qd : qd - o.hi[m];
                    if (box_diff < 0.0f) box_diff = 0.0f;
                    term[l >> 2] = cut_diff * cut_diff - box_diff * box_diff;
                    farm |= 1u << l;
                }
            }
            if (in_lo)
                E = m;
            else
                S = m;
        }
    }
    const int qbase = (threadIdx.x & 63) & ~3;
    farm |= __shfl_xor(farm, 1, 64);
    farm |= __shfl_xor(farm, 2, 64);
    float box = root_box;
    bool ok = true;
#pragma unroll
    for (int l = 0; l < 32; l++) {
        const float t = __shfl(term[l >> 2], qbase + (l & 3), 64);
        if ((farm >> l) & 1) {
            box = box + t;
            ok = ok && box <= D;
        }
    }
    return ok;
}

// ANNkd_leaf's distance with its early break: the sequential fp32 sum of (q_d - p_d)^2 into dist, false once it
// exceeds lim (never inserted).  Summed 8 terms per step with the step's loads issued together and the test after
// the step: the partial sums only grow, so this is false exactly when ANN's per-term test breaks (a NaN sum never
// breaks there either), and the sum is the same.
__device__ __forceinline__ bool kd_leaf_dist(const float *__restrict__ qr, const float *__restrict__ pp, int dd,
                                             float lim, float &dist) {
    dist = 0.0f;
    int d = 0;
    for (; d + 8 <= dd; d += 8) {
        float v[8], w[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            v[u] = pp[d + u];
            w[u] = qr[d + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const float t = w[u] - v[u];
            dist = dist + t * t;
        }
        if (dist > lim) return false;
    }
    for (; d < dd; d++) {
        const float t = qr[d] - pp[d];
        dist = dist + t * t;
        if (dist > lim) return false;
    }
    return true;
}

// annkSearch replayed exactly for one query (kd_search.cpp; ANN.dll 0x1800128e0, ANNkd_split::ann_search 0x180012b60,
// ANNkd_leaf::ann_search 0x180012cf0): depth-first, near child first, far child iff its box distance < the current
// k-th key (eps = 0), leaf scans with the early break, ANNmin_k insertion (equal keys keep the first found).  One
// thread; the explicit stack holds pending nodes and pending far checks.  Writes idx[0..k) / err[0..k) (missing:
// -1 / FLT_MAX) and returns the best index (-1: none).  K >= k.
template <int K>
__device__ int kd_replay_query(const KdOrder &o, const float *__restrict__ rows, const float *__restrict__ qr, int k,
                               int *__restrict__ idx, float *__restrict__ err) {
    float mk[K + 1];
    int mi[K + 1];
    int cnt = 0;
    auto max_key = [&]() { return cnt == k ? mk[k - 1] : FLT_MAX; };
    // stack frames: kind 0 = visit node [s, e) with box b; kind 1 = far check of node [s, e)'s child
    struct Fr {
        int s, e, kind;
        float b;
    };
    Fr st[96];
    int sp = 0;
    st[sp++] = Fr{0, o.n, 0, kd_root_box(o, qr)};
    while (sp > 0) {
        const Fr f = st[--sp];
        if (f.kind == 0) {
            if (f.e - f.s <= o.bs) {  // ANNkd_leaf::ann_search
                float min_dist = max_key();
                for (int p = f.s; p < f.e; p++) {
                    const int pt = o.pidx[p];
                    const float *pp = rows + (long)pt * o.dd;
                    float dist;
                    if (kd_leaf_dist(qr, pp, o.dd, min_dist, dist)) {  // ANNmin_k::insert
                        int i;
                        for (i = cnt; i > 0; i--) {
                            if (mk[i - 1] > dist) {
                                mk[i] = mk[i - 1];
                                mi[i] = mi[i - 1];
                            } else {
                                break;
                            }
                        }
                        mk[i] = dist;
                        mi[i] = pt;
                        if (cnt < k) cnt++;
                        min_dist = max_key();
                    }
                }
                continue;
            }
            const int m = f.s + ((f.e - f.s) >> 1);
            const float cut_diff = qr[o.cd[m]] - o.cv[m];
            // near child now, far check after it returns (pushed first, popped after the near subtree)
            st[sp++] = Fr{f.s, f.e, 1, f.b};
            if (cut_diff < 0.0f)
                st[sp++] = Fr{f.s, m, 0, f.b};
            else
                st[sp++] = Fr{m, f.e, 0, f.b};
        } else {
            const int m = f.s + ((f.e - f.s) >> 1);
            const float qd = qr[o.cd[m]];
            const float cut_diff = qd - o.cv[m];
            const bool lo_first = cut_diff < 0.0f;
            float box_diff = lo_first ? o.lo[m] - qd : qd - o.hi[m];
            if (box_diff < 0.0f) box_diff = 0.0f;
            const float b = f.b + (cut_diff * cut_diff - box_diff * box_diff);
            if (b * 1.0f < max_key()) st[sp++] = lo_first ? Fr{m, f.e, 0, b} : Fr{f.s, m, 0, b};
        }
    }
    for (int j = 0; j < k; j++) {
        const bool ok = j < cnt;
        idx[j] = ok ? mi[j] : -1;
        err[j] = ok ? mk[j] : FLT_MAX;
    }
    return cnt > 0 ? mi[0] : -1;
}

}  // namespace tiler

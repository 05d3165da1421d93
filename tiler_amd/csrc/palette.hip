// palette.hip -- palette generation of the Dither step on the GPU: QuantizePalette with the
// default Dennis Lee v3 quantizer (main.pas:2154-2254, 2396-2433 -> dl3quant, dlquant/quantizer.c:437-663) for
// every (keyframe, palette) pair in one pass, then the CompareCMULHS order of the 16 colours (main.pas:2081-2090,
// 2413) and FinishQuantizePalette's use-count order (main.pas:2435-2480).
//
// GPU layout, all pairs at once (the reference runs one DoQuantize per pair, main.pas:872-875, 901):
//   1. every pixel of every tile -> key (pair << 3*bpc | the bpc-bit colour cell, build_table3's index) and its
//      0x00BBGGRR value; a radix sort by key + reduce-by-key gives every pair's CUBE3 table in index order with
//      32-bit wrapping sums (MSVC `ulong`, as the reference DLL) -- the tile order does not matter to a histogram;
//   2. pass 1 of reduce_table3 (recount_next for every entry: the O(n^2 / 2) nearest-merge search) with one wave
//      per entry over the whole grid;
//   3. pass 2 (the sequential merges) with one 1024-thread workgroup per pair: each merge is the minimum error
//      over chunk minima, one pass over the table that applies every entry's fix-ups (re-point, the updates of
//      recount_dist(c1) and recount_dist(c2)) or lists it for recount_next, and one batched, load-balanced scan
//      for all listed recount_next; results are those of the sequential loops because each entry's steps only
//      depend on its own state and on table data the merge does not change (dl3_merge_pass).
// calc_err is evaluated exactly as quantizer.c:512-541 in IEEE single precision: integer cell means, squares of
// integers (exact), sqrt through double (innocuous for sqrt: 53 >= 2 * 24 + 2) rounded once to float.
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "palette.hpp"
#include "tiler_common.hpp"

namespace tiler {

namespace {

constexpr int DL3_T = 1024;        // pass-2 workgroup
constexpr int DL3_W = DL3_T / 64;  // its waves

struct Dl3Sum {
    uint32_t r, g, b, n;
};

struct Dl3SumOp {
    __host__ __device__ Dl3Sum operator()(const Dl3Sum &a, const Dl3Sum &b) const {
        return Dl3Sum{a.r + b.r, a.g + b.g, a.b + b.b, a.n + b.n};
    }
};

struct Dl3Expand {  // one pixel 0x00BBGGRR -> its CUBE3 contribution (build_table3, quantizer.c:496-499)
    __host__ __device__ Dl3Sum operator()(const uint32_t c) const {
        return Dl3Sum{c & 255u, (c >> 8) & 255u, (c >> 16) & 255u, 1u};
    }
};

// the colour tables of all pairs; entry e of pair p at seg[p] + local index, split by access: the nearest-merge
// scans read QN alone (8 bytes per entry), the per-merge pass QN and EC, calc_err also V.
struct Dl3Tab {
    uint2 *QN;  // x = Q (rr | gg << 8 | bb << 16, setrgb), y = (float)N, bits (the scans' bounds; V.w is exact)
    uint2 *EC;  // x = E (err, float bits), y = C (cc)
    uint4 *V;   // x, y, z = CUBE3 r, g, b (32-bit, wrapping); w = N
};
#ifndef DL3_U_V
#define DL3_U_V 6
#endif
#ifndef DL3_UM_V
#define DL3_UM_V 4
#endif
#ifndef DL3_PROBE
#define DL3_PROBE 1  // recount: each listed entry's first 64 candidates before the bulk scan (0: A/B builds only)
#endif
constexpr int DL3_U = DL3_U_V;    // records loaded per lane before any is used
constexpr int DL3_UM = DL3_UM_V;  // the same in the merge pass (two records per entry)
// the scans load up to 64 * unroll + 63 records past tot, into the QN / EC tables' 1,024-record slack
static_assert(64 * (DL3_U + 1) <= 1024 && 64 * (DL3_UM + 1) <= 1024, "DLv3 unroll depth exceeds the table slack");

__device__ __forceinline__ void dl3_set_ec(const Dl3Tab &t, int i, float e, int c) {
    t.EC[i] = make_uint2(__float_as_uint(e), (uint32_t)c);
}

__device__ __forceinline__ uint32_t dl3_setrgb(uint32_t r, uint32_t g, uint32_t b, uint32_t n) {  // quantizer.c:472-478
    const int v = (int)n, v2 = v >> 1;
    const uint32_t rr = (uint8_t)((r + (uint32_t)v2) / (uint32_t)v);
    const uint32_t gg = (uint8_t)((g + (uint32_t)v2) / (uint32_t)v);
    const uint32_t bb = (uint8_t)((b + (uint32_t)v2) / (uint32_t)v);
    return rr | (gg << 8) | (bb << 16);
}

__device__ __forceinline__ float dl3_sq(int d) { return (float)(d * d); }  // squares3[d] (exact for |d| <= 255)

__device__ __forceinline__ float dl3_sqrt(float x) { return (float)__builtin_sqrt((double)x); }

struct Dl3Entry {
    uint32_t r, g, b, n, q;
};

__device__ __forceinline__ uint2 dl3_qn(uint32_t q, uint32_t n) { return make_uint2(q, __float_as_uint((float)n)); }

__device__ __forceinline__ Dl3Entry dl3_entry(uint32_t q, const uint4 &v) { return Dl3Entry{v.x, v.y, v.z, v.w, q}; }

__device__ __forceinline__ Dl3Entry dl3_load(const Dl3Tab &t, int i) { return dl3_entry(t.QN[i].x, t.V[i]); }

__device__ __forceinline__ float dl3_calc_err(const Dl3Entry &a, const Dl3Entry &b) {  // quantizer.c:512-541
    const uint32_t P1 = a.n, P2 = b.n, P3 = P1 + P2;
    const int R3 = (int)((a.r + b.r + (P3 >> 1)) / P3);
    const int G3 = (int)((a.g + b.g + (P3 >> 1)) / P3);
    const int B3 = (int)((a.b + b.b + (P3 >> 1)) / P3);
    const int R1 = a.q & 255, G1 = (a.q >> 8) & 255, B1 = (a.q >> 16) & 255;
    const int R2 = b.q & 255, G2 = (b.q >> 8) & 255, B2 = (b.q >> 16) & 255;
    float d1 = dl3_sq(R3 - R1) + dl3_sq(G3 - G1) + dl3_sq(B3 - B1);
    d1 = dl3_sqrt(d1) * (float)P1;
    float d2 = dl3_sq(R2 - R3) + dl3_sq(G2 - G3) + dl3_sq(B2 - B3);
    d2 = dl3_sqrt(d2) * (float)P2;
    return d1 + d2;
}

// True when the COMPUTED calc_err(a, b) is certainly > e, so the candidate can neither win nor tie.  The exact value
// is >= m * |Q_a - Q_b| with m = min(P_a, P_b) (sqrt(d1) + sqrt(d2) >= |Q_a - Q_b|, the triangle inequality through
// the merged mean), the float evaluation loses at most (1 - 2^-24)^5, so computed^2 >= m^2 * dd * (1 - 6e-7).  The
// test's own float evaluation (dd exact, m rounded once, three products, e * e) is within (1 +- 2^-24)^6, so with
// the factor 1 - 1e-5 a true result implies computed^2 > e^2.  e = inf (or e * e overflowing) never prunes.
__device__ __forceinline__ bool dl3_cannot(uint32_t qa, float na, uint32_t qb, float nb, float e) {
    const int dr = (int)(qa & 255) - (int)(qb & 255), dg = (int)((qa >> 8) & 255) - (int)((qb >> 8) & 255);
    const int db = (int)((qa >> 16) & 255) - (int)((qb >> 16) & 255);
    const float m = fminf(na, nb);  // the counts as floats: rounded once each, as the margin allows
    return (float)(dr * dr + dg * dg + db * db) * m * m * 0.99999f > e * e;
}

// The scans' first test, cheaper than dl3_cannot: |Q_a - Q_b|_2 >= |Q_a - Q_b|_1 / sqrt(3) (three channels), and the L1
// distance of the packed bytes is one v_sad_u8.  e3 = e * e * 3.00003 (dl3_e3); L1 (<= 765) converts exactly, m is
// rounded once, so a true result implies (m * L1)^2 / 3 > e^2 (1 + 9e-6) and, as for dl3_cannot, computed calc_err > e.
__device__ __forceinline__ float dl3_e3(float e) { return e * e * 3.00003f; }
__device__ __forceinline__ bool dl3_cannot_l1(uint32_t qa, float na, uint32_t qb, float nb, float e3) {
    const float t = (float)__builtin_amdgcn_sad_u8(qa, qb, 0u) * fminf(na, nb);
    return t * t > e3;
}

// first minimum: smaller error, equal errors -> smaller index (the reference's ascending scan with `<`)
__device__ __forceinline__ void dl3_min(float &e, int &j, float e2, int j2) {
    if (e2 < e || (e2 == e && j2 < j)) {
        e = e2;
        j = j2;
    }
}

__device__ __forceinline__ void dl3_wave_min(float &e, int &j) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float e2 = __shfl_xor(e, o);
        const int j2 = __shfl_xor(j, o);
        dl3_min(e, j, e2, j2);
    }
}

// block-wide first minimum; every thread returns the result
__device__ void dl3_block_min(float &e, int &j, float *sh_e, int *sh_j) {
    dl3_wave_min(e, j);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // sh_* free (a previous call's readers are done)
    if ((threadIdx.x & 63) == 0) {
        sh_e[w] = e;
        sh_j[w] = j;
    }
    __syncthreads();
    e = sh_e[0];
    j = sh_j[0];
    for (int k = 1; k < DL3_W; k++) dl3_min(e, j, sh_e[k], sh_j[k]);
}

// Chunk minima of the error column, so each merge's "first entry of minimum error" scans one value per chunk
// instead of the whole table: every write of err[i] (and every entry moved or removed) marks its chunk, and the
// marked chunks are recomputed at the end of the merge.  A chunk's value is its first minimum (smallest error,
// then smallest index), so the minimum over chunks is the reference's first minimum.
constexpr int DL3_MAXCH = 4096;
struct Dl3Chunks {
    float e[DL3_MAXCH];
    int j[DL3_MAXCH];
    int c[DL3_MAXCH];  // cc of entry j (so the merge's c2 needs no table read)
    unsigned bits[DL3_MAXCH / 32];
    int dirty[DL3_MAXCH];
    int n, sh;  // dirty count; log2 of the chunk size
};

__device__ __forceinline__ void dl3_mark(Dl3Chunks *ch, int i) {
    const int c = i >> ch->sh;
    const unsigned m = 1u << (c & 31);
    if (!(atomicOr(&ch->bits[c >> 5], m) & m)) ch->dirty[atomicAdd(&ch->n, 1)] = c;
}

// recount_next(i) (quantizer.c:543-560) by one wave over j in (i, tot): each lane's first minimum (its j ascend,
// `<` keeps the earlier of equal errors), then the wave's; lane 0 stores it (cc = 0 for an empty range)
__device__ void dl3_recount_wave(const Dl3Tab &t, int i, int tot) {
    const Dl3Entry a = dl3_load(t, i);
    float e = HUGE_VALF;
    int j = INT32_MAX;
    const int lane = (int)(threadIdx.x & 63);
    for (int k0 = i + 1 + lane; k0 < tot; k0 += 64 * DL3_U) {
        uint2 r[DL3_U];
        const uint2 *p = t.QN + k0;  // loads past tot stay inside the table allocation (its slack)
#pragma unroll
        for (int u = 0; u < DL3_U; u++) r[u] = p[u * 64];
        const float e3 = dl3_e3(e), naf = (float)a.n;
#pragma unroll
        for (int u = 0; u < DL3_U; u++) {
            const int k = k0 + u * 64;
            const float nb = __uint_as_float(r[u].y);
            if (k >= tot || dl3_cannot_l1(a.q, naf, r[u].x, nb, e3) || dl3_cannot(a.q, naf, r[u].x, nb, e))
                continue;
            const float cur = dl3_calc_err(a, dl3_entry(r[u].x, t.V[k]));
            if (cur < e) {
                e = cur;
                j = k;
            }
        }
    }
    dl3_wave_min(e, j);
    if (lane == 0) dl3_set_ec(t, i, e, j == INT32_MAX ? 0 : j);
}

// ---------------------------------------------------------------------------------------------------------------
// 1. keys / values of every pixel; tiles per pair (PaletteUseCount)
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dl3_keys_kernel(const int32_t *__restrict__ rgb, const int32_t *__restrict__ pal_of,
                                                       const uint8_t *__restrict__ active, long n_tiles, int P, int bpc,
                                                       uint32_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                       int *__restrict__ use_count) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_tiles * 64) return;
    const long tile = i >> 6;
    const int p = pal_of[tile];
    const bool ok = (!active || active[tile]) && p >= 0 && p < P;
    const uint32_t c = (uint32_t)rgb[i];
    const int mbpc = (1 << bpc) - 1;
    const uint32_t r = (c & 255u) * mbpc / 255, g = ((c >> 8) & 255u) * mbpc / 255, b = ((c >> 16) & 255u) * mbpc / 255;
    keys[i] = ok ? ((uint32_t)p << (3 * bpc)) | b | (g << bpc) | (r << (2 * bpc)) : ((uint32_t)P << (3 * bpc));
    vals[i] = c;
    if (ok && (i & 63) == 0) atomicAdd(use_count + p, 1);
}

// seg[p] = first entry of pair p (lower bound of p << 3*bpc in the sorted unique keys), seg[P] = entries
__global__ void dl3_seg_kernel(const uint32_t *__restrict__ ukeys, const int *__restrict__ nruns, int P, int bpc,
                               int *__restrict__ seg) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p > P) return;
    const uint32_t key = (uint32_t)p << (3 * bpc);
    int lo = 0, hi = *nruns;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ukeys[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    seg[p] = lo;
}

__global__ __launch_bounds__(256) void dl3_init_kernel(const Dl3Sum *__restrict__ agg, const int *__restrict__ seg, int P,
                                                       Dl3Tab t) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= seg[P]) return;
    const Dl3Sum s = agg[e];
    t.V[e] = make_uint4(s.r, s.g, s.b, s.n);
    t.QN[e] = dl3_qn(dl3_setrgb(s.r, s.g, s.b, s.n), s.n);  // EC: pass 1
}

// ---------------------------------------------------------------------------------------------------------------
// 2. pass 1 of reduce_table3 (quantizer.c:589-599): recount_next(i) for every entry, one wave per entry
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dl3_pass1_kernel(const uint32_t *__restrict__ ukeys, const int *__restrict__ seg,
                                                        int P, int bpc, Dl3Tab t) {
    const int total = seg[P];
    for (int e = blockIdx.x * 4 + (threadIdx.x >> 6); e < total; e += gridDim.x * 4) {
        const int p = (int)(ukeys[e] >> (3 * bpc));
        const int s = seg[p], n = seg[p + 1] - s, i = e - s;
        Dl3Tab u = t;
        u.QN += s, u.EC += s, u.V += s;
        if (i == n - 1) {  // the last entry (quantizer.c:598-599)
            if ((threadIdx.x & 63) == 0) dl3_set_ec(u, i, HUGE_VALF, n);
        } else {
            dl3_recount_wave(u, i, n);
        }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// 3. pass 2 of reduce_table3 (quantizer.c:603-643): one workgroup per pair, the merges in order
// ---------------------------------------------------------------------------------------------------------------
struct Dl3Args {
    Dl3Tab t;
    const int *seg;
    int quant_to;
    int *list;       // [entries] recount-list overflow (a pair's slice at its seg offset)
    int lcap;        // recount-list entries held in LDS per batch (DL3_LCAP; smaller only by the test hook)
    int32_t *pal;    // [P][quant_to] 0x00BBGGRR
};


// One merge's recount list, batched: every listed entry's recount_next scan is cut into units of 64 candidates,
// the units of the whole batch are split evenly over the waves, and each candidate that survives the bound is
// folded into its entry's slot by a 64-bit LDS atomic minimum of (err bits, index) -- the first minimum, as err >= 0
// orders like its bits.  Every scan reads only table data no step of the merge writes (QN, V), so the order of the
// candidates does not matter, and the slot's current value is an achieved error, hence a valid pruning bound.
constexpr int DL3_LCAP = 1024;
constexpr unsigned long long DL3_NONE = (0x7f800000ull << 32) | 0xffffffffull;  // (inf, no index)
struct Dl3List {
    int item[DL3_LCAP];
    int n;  // listed entries (those >= lcap in the global overflow)
};
struct Dl3Batch {  // the batched recount's per-item state
    uint2 qn[DL3_LCAP];
    uint4 v[DL3_LCAP];
    unsigned long long slot[DL3_LCAP];
    int pre[DL3_LCAP + 1];  // exclusive prefix of the items' unit counts
    int wsum[DL3_W];
};

__device__ __forceinline__ void dl3_push(Dl3List *L, int *glist, int i, int lcap) {
    const int k = atomicAdd(&L->n, 1);
    if (k < lcap)
        L->item[k] = i;
    else
        glist[k] = i;
}

struct Dl3Merge {  // one merge's fix-up context
    int c1, c2, tot;
    bool c2v;
    Dl3Entry b1, b2;  // the new c1 and c2
};

__device__ void dl3_recount_list(const Dl3Tab &t, Dl3List *L, Dl3Batch *B, const int *glist, int K, int tot,
                                 Dl3Chunks *ch, int lcap, const Dl3Merge &m) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int base = 0; base < K; base += lcap) {
        const int nb = min(lcap, K - base);
        int units = 0;
        if (tid < nb) {
            const int i = base ? glist[base + tid] : L->item[tid];
            if (base) L->item[tid] = i;  // the previous batch's readers passed its last barrier
            const uint2 qn = t.QN[i];
            const uint4 v = t.V[i];
            B->qn[tid] = qn;
            B->v[tid] = v;
            // the slot starts at the merge's new entries when they lie in (i, tot): candidates like any other (so
            // the result is unchanged), and the merged c2 is usually near what i pointed at, so the scan prunes from
            // its first candidate on
            unsigned long long k0 = DL3_NONE;
            const Dl3Entry ai = dl3_entry(qn.x, v);
            if (m.c2v && m.c2 > i) {
                const unsigned long long k = ((unsigned long long)__float_as_uint(dl3_calc_err(ai, m.b2)) << 32) | (uint32_t)m.c2;
                k0 = k < k0 ? k : k0;
            }
            if (m.c1 > i) {
                const unsigned long long k = ((unsigned long long)__float_as_uint(dl3_calc_err(ai, m.b1)) << 32) | (uint32_t)m.c1;
                k0 = k < k0 ? k : k0;
            }
            B->slot[tid] = k0;
            units = (tot - 1 - i + 63) >> 6;
        }
        int v = units;  // block-wide exclusive scan of the unit counts
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int x = __shfl_up(v, o);
            if (lane >= o) v += x;
        }
        if (lane == 63) B->wsum[w] = v;
        __syncthreads();
        int off = 0;
        for (int k = 0; k < w; k++) off += B->wsum[k];
        if (tid < nb) B->pre[tid + 1] = off + v;
        if (tid == 0) B->pre[0] = 0;
        __syncthreads();
        const int U = B->pre[nb];
        const int ua = (int)((long)U * w / DL3_W), ub = (int)((long)U * (w + 1) / DL3_W);
        int q = 0;  // the item of unit ua: the last q with pre[q] <= ua
        for (int lo = 0, hi = nb; lo < hi;) {
            const int mid = (lo + hi + 1) >> 1;
            if (B->pre[mid] <= ua) {
                lo = mid;
                q = mid;
            } else {
                hi = mid - 1;
            }
        }
        // the wave's units item by item, up to DL3_U units a step: the item, its bound and the step's shape are
        // wave-uniform; per candidate one load, the L1 test (dl3_cannot_l1), and for the few that pass it the exact
        // bound and calc_err.  The scan's VALU is what bounds it (a 64-lane op issues over 4 cycles).
#if DL3_PROBE
        // probe: every item's first unit (its next 64 entries: neighbours in the table's colour-cell order, so
        // usually close) scanned first, one wave per item, so the slots hold a tight bound before the bulk scan
        for (int qq = w; qq < nb; qq += DL3_W) {
            const int u0 = B->pre[qq];
            if (u0 >= B->pre[qq + 1]) continue;  // empty range (uniform)
            const int j = L->item[qq] + 1 + lane;
            const uint2 rr = t.QN[j];
            const uint2 a = B->qn[qq];
            const float naf = __uint_as_float(a.y), eb = __uint_as_float((uint32_t)(B->slot[qq] >> 32));
            const float nb2 = __uint_as_float(rr.y);
            if (j < tot && !dl3_cannot_l1(a.x, naf, rr.x, nb2, dl3_e3(eb)) && !dl3_cannot(a.x, naf, rr.x, nb2, eb)) {
                const float cur = dl3_calc_err(dl3_entry(a.x, B->v[qq]), dl3_entry(rr.x, t.V[j]));
                if (cur <= eb) atomicMin(&B->slot[qq], ((unsigned long long)__float_as_uint(cur) << 32) | (uint32_t)j);
            }
        }
        __syncthreads();
#endif
        for (int u0 = ua; u0 < ub;) {
            while (q < nb - 1 && B->pre[q + 1] <= u0) q++;
#if DL3_PROBE
            if (u0 == B->pre[q]) {  // the probed unit
                u0++;
                continue;
            }
#endif
            const int nu = min(DL3_U, min(ub, B->pre[q + 1]) - u0);
            const int j0 = L->item[q] + 1 + ((u0 - B->pre[q]) << 6) + lane;
            uint2 r[DL3_U];
            const uint2 *pj = t.QN + j0;  // one address, immediate offsets; loads past tot stay inside the slack
#pragma unroll
            for (int u = 0; u < DL3_U; u++) r[u] = pj[u << 6];
            const uint2 a = B->qn[q];
            const float naf = __uint_as_float(a.y);
            float eb = __uint_as_float((uint32_t)(B->slot[q] >> 32));
            float e3 = dl3_e3(eb);
#pragma unroll
            for (int u = 0; u < DL3_U; u++) {
                const int j = j0 + (u << 6);
                const float nb = __uint_as_float(r[u].y);
                if (u >= nu || j >= tot || dl3_cannot_l1(a.x, naf, r[u].x, nb, e3)) continue;
                if (dl3_cannot(a.x, naf, r[u].x, nb, eb)) continue;
                const float cur = dl3_calc_err(dl3_entry(a.x, B->v[q]), dl3_entry(r[u].x, t.V[j]));
                if (cur <= eb) {
                    atomicMin(&B->slot[q], ((unsigned long long)__float_as_uint(cur) << 32) | (uint32_t)j);
                    eb = cur;  // an achieved value: still a valid bound for this lane
                    e3 = dl3_e3(eb);
                }
            }
            u0 += nu;
        }
        __syncthreads();
        if (tid < nb) {
            const unsigned long long k = B->slot[tid];
            const int i = L->item[tid];
            dl3_set_ec(t, i, __uint_as_float((uint32_t)(k >> 32)), (uint32_t)k == 0xffffffffu ? 0 : (int)(uint32_t)k);
            dl3_mark(ch, i);
        }
        __syncthreads();
    }
}

// the first minimum of chunk c over entries below tot, by one wave (lane 0 stores it)
__device__ void dl3_chunk_min(const Dl3Tab &t, Dl3Chunks *ch, int c, int tot) {
    const int b = c << ch->sh, e = min(tot, b + (1 << ch->sh));
    float v = HUGE_VALF;
    int j = INT32_MAX, cc = 0;
    for (int i0 = b + (int)(threadIdx.x & 63); i0 < e; i0 += 64 * DL3_U) {
        uint2 r[DL3_U];
#pragma unroll
        for (int u = 0; u < DL3_U; u++) r[u] = t.EC[min(i0 + u * 64, e - 1)];
#pragma unroll
        for (int u = 0; u < DL3_U; u++) {
            const float x = __uint_as_float(r[u].x);
            if (i0 + u * 64 < e && x < v) {
                v = x;
                j = i0 + u * 64;
                cc = (int)r[u].y;
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {  // dl3_wave_min carrying the winner's cc
        const float v2 = __shfl_xor(v, o);
        const int j2 = __shfl_xor(j, o), c2 = __shfl_xor(cc, o);
        if (v2 < v || (v2 == v && j2 < j)) {
            v = v2;
            j = j2;
            cc = c2;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        ch->e[c] = v;
        ch->j[c] = j;
        ch->c[c] = cc;
    }
}


// entry i's fix-ups (qn, ec: its QN and EC; getv() its V): the list, or the updates written
template <class GetV>
__device__ __forceinline__ void dl3_fixup(const Dl3Tab &t, Dl3List *L, int *glist, int lcap, Dl3Chunks *ch,
                                          const Dl3Merge &m, int i, uint2 qn, uint2 ec, GetV getv) {
    int c = (int)ec.y;
    float e = __uint_as_float(ec.x);
    bool rc = false, wr = false;
    if (i == m.c1) {
        rc = true;
    } else if (i > m.c1) {
        rc = c == m.tot;
    } else {
        if (c == m.tot) {
            c = m.c1;
            wr = true;
        }
        if (c == m.c1) {
            rc = true;
        } else if (!dl3_cannot_l1(m.b1.q, (float)m.b1.n, qn.x, __uint_as_float(qn.y), dl3_e3(e)) &&
                   !dl3_cannot(qn.x, __uint_as_float(qn.y), m.b1.q, (float)m.b1.n, e)) {
            const float cur = dl3_calc_err(dl3_entry(qn.x, getv()), m.b1);
            if (cur < e) {
                e = cur;
                c = m.c1;
                wr = true;
            }
        }
    }
    if (!rc && m.c2v && i <= m.c2) {
        if (i == m.c2 || c == m.c2) {
            rc = true;
        } else if (!dl3_cannot_l1(m.b2.q, (float)m.b2.n, qn.x, __uint_as_float(qn.y), dl3_e3(e)) &&
                   !dl3_cannot(qn.x, __uint_as_float(qn.y), m.b2.q, (float)m.b2.n, e)) {
            const float cur = dl3_calc_err(dl3_entry(qn.x, getv()), m.b2);
            if (cur < e) {
                e = cur;
                c = m.c2;
                wr = true;
            }
        }
    }
    if (rc) {
        dl3_push(L, glist, i, lcap);
    } else if (wr) {
        dl3_set_ec(t, i, e, c);
        dl3_mark(ch, i);
    }
}

// One merge's fix-ups (quantizer.c:631-642) as one pass with each entry in its own lane.  The reference's loops --
// re-point i < c1 from the moved entry to c1; recount_next(i) for i > c1 pointing at it; recount_dist(c1); then
// recount_dist(c2) unless c2 was the last entry -- only ever change entry i from entry i's own state and table data
// none of them writes (QN, V are final once the merge is applied), so each entry's sequence of steps can run on its
// own.  A recount_next makes every later step of the same entry a no-op: its scan over (i, tot) already covers c1
// and c2 whenever a later step would compare against them (c1 < c2, and those steps only visit i < c1 or i < c2),
// and a repeated recount gives the same result.  So an entry either joins the recount list, or takes the updates
// with calc_err(i, c1) then calc_err(i, c2) (strictly smaller only, as the reference).
__device__ void dl3_merge_pass(const Dl3Tab &t, Dl3List *L, int *glist, const Dl3Merge &m, Dl3Chunks *ch, int lcap) {
    const int tot = m.tot, lane = threadIdx.x & 63;
    // wave-contiguous blocks of 64 * DL3_UM entries (one address per block, immediate offsets; loads past tot stay
    // inside the tables' slack), blocks round robin over the waves
    for (int i0 = (int)(threadIdx.x >> 6) * 64 * DL3_UM + lane; i0 < tot; i0 += DL3_T * DL3_UM) {
        uint2 rq[DL3_UM], re[DL3_UM];
        const uint2 *pq = t.QN + i0, *pe = t.EC + i0;
#pragma unroll
        for (int u = 0; u < DL3_UM; u++) {
            rq[u] = pq[u * 64];
            re[u] = pe[u * 64];
        }
#pragma unroll
        for (int u = 0; u < DL3_UM; u++) {
            const int i = i0 + u * 64;
            if (i >= tot) break;
            dl3_fixup(t, L, glist, lcap, ch, m, i, rq[u], re[u], [&]() { return t.V[i]; });
        }
    }
}


__global__ __launch_bounds__(DL3_T) void dl3_reduce_kernel(Dl3Args a) {
    __shared__ float sh_e[DL3_W];
    __shared__ int sh_j[DL3_W];
    __shared__ Dl3Chunks chs;
    __shared__ Dl3List lst;
    __shared__ Dl3Merge sm;  // this merge's c1, c2 and their new entries (thread 0 -> everyone)
    __shared__ Dl3Batch bat;
    Dl3Chunks *ch = &chs;
    Dl3List *L = &lst;
    Dl3Batch *B = &bat;
    const int p = blockIdx.x;
    const int s = a.seg[p], n = a.seg[p + 1] - s;
    if (n <= a.quant_to) {  // nothing to merge
        for (int i = threadIdx.x; i < a.quant_to; i += DL3_T)
            a.pal[(long)p * a.quant_to + i] = i < n ? (int32_t)a.t.QN[s + i].x : 0;
        return;
    }
    Dl3Tab t = a.t;
    t.QN += s, t.EC += s, t.V += s;
    int *glist = a.list + s;
    int sh = 0;
    while (((n + (1 << sh) - 1) >> sh) > DL3_MAXCH) sh++;
    if (threadIdx.x == 0) {
        ch->n = 0;
        ch->sh = sh;
    }
    for (int w = threadIdx.x; w < DL3_MAXCH / 32; w += DL3_T) ch->bits[w] = 0;
    __syncthreads();
    for (int c = threadIdx.x >> 6; c < ((n + (1 << sh) - 1) >> sh); c += DL3_W) dl3_chunk_min(t, ch, c, n);
    __syncthreads();
    int tot = n, c1 = 0;
    while (tot > a.quant_to) {
        // the first entry of minimum error (quantizer.c:610-618) over the chunk minima; none below HUGE_VALF
        // keeps c1
        float e = HUGE_VALF;
        int j = INT32_MAX;
        const int nch = (tot + (1 << sh) - 1) >> sh;
        for (int c = threadIdx.x; c < nch; c += DL3_T) dl3_min(e, j, ch->e[c], ch->j[c]);
        dl3_block_min(e, j, sh_e, sh_j);
        int c2;
        if (j != INT32_MAX) {
            c1 = j;
            c2 = ch->c[j >> sh];  // the chunk minimum's cc
        } else {
            c2 = (int)t.EC[c1].y;
        }
        __syncthreads();  // every thread has read the chunk minima before they change
        tot--;
        if (threadIdx.x == 0) {  // merge c1 into c2, the last entry into c1 (quantizer.c:619-629): one round of loads
            const uint32_t ql = t.QN[tot].x;
            const uint4 v1 = t.V[c1], v2 = t.V[c2], vl = t.V[tot];
            const uint2 el = t.EC[tot];
            const uint32_t r = v2.x + v1.x, g = v2.y + v1.y, b = v2.z + v1.z, nn = v2.w + v1.w;
            const uint32_t qm = dl3_setrgb(r, g, b, nn);
            const uint4 vm = make_uint4(r, g, b, nn);
            t.V[c2] = vm;
            t.QN[c2] = dl3_qn(qm, nn);
            // the last entry moves into c1 (after the c2 update: c2 may be the last entry)
            const bool c2last = c2 == tot;
            const uint32_t qc1 = c2last ? qm : ql;
            const uint4 vc1 = c2last ? vm : vl;
            t.V[c1] = vc1;
            t.QN[c1] = dl3_qn(qc1, vc1.w);
            t.EC[c1] = el;
            dl3_set_ec(t, tot - 1, HUGE_VALF, tot);
            L->n = 0;
            sm.c1 = c1;
            sm.c2 = c2;
            sm.tot = tot;
            sm.c2v = !c2last;
            sm.b1 = dl3_entry(qc1, vc1);
            sm.b2 = c2last ? sm.b1 : dl3_entry(qm, vm);
            dl3_mark(ch, c1);
            dl3_mark(ch, tot - 1);
            dl3_mark(ch, tot);  // the removed entry leaves its chunk
        }
        __syncthreads();
        {
            const Dl3Merge m = sm;
            dl3_merge_pass(t, L, glist, m, ch, a.lcap);
        }
        __syncthreads();
        dl3_recount_list(t, L, B, glist, L->n, tot, ch, a.lcap, sm);
        // refresh the marked chunks (every mark above is complete: the list run ends in a barrier)
        const int nd = ch->n;
        for (int q = threadIdx.x >> 6; q < nd; q += DL3_W) dl3_chunk_min(t, ch, ch->dirty[q], tot);
        __syncthreads();
        for (int q = threadIdx.x; q < nd; q += DL3_T) ch->bits[ch->dirty[q] >> 5] = 0;
        if (threadIdx.x == 0) ch->n = 0;
        __syncthreads();
    }
    for (int i = threadIdx.x; i < a.quant_to; i += DL3_T)  // set_palette3 + copy_pal (calloc'd beyond tot)
        a.pal[(long)p * a.quant_to + i] = i < tot ? (int32_t)t.QN[i].x : 0;
}

// ---------------------------------------------------------------------------------------------------------------
// host: CompareCMULHS (TFPList.Sort) and FinishQuantizePalette's order
// ---------------------------------------------------------------------------------------------------------------
}  // namespace

static std::atomic<int> g_dl3_lcap{DL3_LCAP};  // tiler_debug_dl3
void dl3_debug(int list_cap) {
    g_dl3_lcap.store(list_cap > 0 ? list_cap : DL3_LCAP);
}

namespace {

int muldiv_win(int a, int b, int c) {  // Windows MulDiv (unit windows in main.pas's uses): rounded half away from 0
    if (c == 0) return -1;
    if (c < 0) {
        a = -a;
        c = -c;
    }
    const long long prod = (long long)a * b;
    const bool add = (a < 0 && b < 0) || (a >= 0 && b >= 0);  // the operands' signs pick the rounding direction
    const long long r = add ? (prod + c / 2) / c : (prod - c / 2) / c;
    if (r > 2147483647LL || r < -2147483647LL) return -1;
    return (int)r;
}

struct CmItem {  // TCountIndexArray (main.pas:193-196)
    int index, luma;
    uint8_t hue, sat, val;
};

CmItem cm_item(int32_t col) {  // FColorMap / FColorMapLuma (main.pas:4835-4847) + RGBToHSV (main.pas:3496-3543)
    const int rr = col & 255, gg = (col >> 8) & 255, bb = (col >> 16) & 255;
    const int mx = std::max(rr, std::max(gg, bb)), mn = std::min(rr, std::min(gg, bb));
    int hh = 0, ss = 0;
    if (mx != mn) {
        const int delta = mx - mn;
        ss = muldiv_win(delta, 255, mx);
        if (rr == mx)
            hh = muldiv_win(42, gg - bb, delta);
        else if (gg == mx)
            hh = muldiv_win(42, bb - rr, delta) + 84;
        else
            hh = muldiv_win(42, rr - gg, delta) + 168;
        hh %= 252;
    }
    CmItem it;
    it.index = col;
    it.luma = (rr * 2126 + gg * 7152 + bb * 722) / 10000;
    it.hue = (uint8_t)(hh & 255);
    it.sat = (uint8_t)(ss & 255);
    it.val = (uint8_t)(mx & 255);
    return it;
}

int cmp3(int a, int b) { return a < b ? -1 : a > b ? 1 : 0; }

int compare_cmulhs(const CmItem *a, const CmItem *b) {  // main.pas:2081-2090
    int r = cmp3(a->luma, b->luma);
    if (!r) r = cmp3(a->val, b->val);
    if (!r) r = cmp3(a->sat, b->sat);
    if (!r) r = cmp3(a->hue, b->hue);
    return r;
}

void fpc_tlist_sort(std::vector<const CmItem *> &l, int L, int R) {  // TFPList.Sort: the FPC RTL QuickSort
    int I, J;
    do {
        I = L;
        J = R;
        const CmItem *P = l[(L + R) / 2];
        do {
            while (compare_cmulhs(P, l[I]) > 0) I++;
            while (compare_cmulhs(P, l[J]) < 0) J--;
            if (I <= J) {
                std::swap(l[I], l[J]);
                I++;
                J--;
            }
        } while (I <= J);
        if (L < J) fpc_tlist_sort(l, L, J);
        L = I;
    } while (I < R);
}

}  // namespace

void sort_palette_cmulhs(int32_t *pal, int n) {
    std::vector<CmItem> items(n);
    std::vector<const CmItem *> l(n);
    for (int i = 0; i < n; i++) {
        items[i] = cm_item(pal[i]);
        l[i] = &items[i];
    }
    if (n > 1) fpc_tlist_sort(l, 0, n - 1);
    std::vector<int32_t> out(n);
    for (int i = 0; i < n; i++) out[i] = l[i]->index;
    memcpy(pal, out.data(), n * sizeof(int32_t));
}

void finish_quantize_order(const int32_t *use_count, int P, int32_t *lut) {
    // kmodes.pas:89-136 QuickSort of the PaletteUseCount records, ComparePaletteUseCount (descending use count)
    std::vector<std::pair<int32_t, int32_t>> a(P);  // (UseCount, PalIdx)
    for (int p = 0; p < P; p++) a[p] = {use_count[p], p};
    auto cmp = [](const std::pair<int32_t, int32_t> &x, const std::pair<int32_t, int32_t> &y) {
        return cmp3(y.first, x.first);
    };
    struct Rec {
        static void qs(std::vector<std::pair<int32_t, int32_t>> &v, int first, int last, decltype(cmp) &c) {
            if (last <= first) return;
            int i, j;
            do {
                i = first;
                j = last;
                int piv = (first + last) >> 1;
                do {
                    while (c(v[i], v[piv]) < 0) i++;
                    while (c(v[j], v[piv]) > 0) j--;
                    if (i <= j) {
                        std::swap(v[i], v[j]);
                        if (piv == i)
                            piv = j;
                        else if (piv == j)
                            piv = i;
                        i++;
                        j--;
                    }
                } while (i <= j);
                if (first < j) qs(v, first, j, c);
                first = i;
            } while (i < last);
        }
    };
    Rec::qs(a, 0, P - 1, cmp);
    for (int p = 0; p < P; p++) lut[a[p].second] = p;
}

// ---------------------------------------------------------------------------------------------------------------
// QuantizePalette for all pairs: device inputs, host outputs
// ---------------------------------------------------------------------------------------------------------------
int quantize_palettes_dev(long n_tiles, const int32_t *d_rgb, const int32_t *d_pal_of, const uint8_t *d_active, int P,
                          int palsize, int bpc, int32_t *pal_out, int32_t *use_count, int32_t *hist,
                          hipStream_t stream) {
    if (n_tiles < 0 || P <= 0 || palsize <= 0 || bpc < 1 || bpc > 8 || (n_tiles > 0 && (!d_rgb || !d_pal_of)) ||
        !pal_out || !use_count) {
        set_error("quantize_palettes: invalid arguments (bpc in 1..8)");
        return -1;
    }
    const int key_bits = 3 * bpc;
    if ((((uint64_t)P + 1) << key_bits) > 0xffffffffull || n_tiles * 64 > 0x7fffffffL) {
        set_error("quantize_palettes: too many palettes for 32-bit keys at this bpc, or more than 2^31 pixels");
        return -1;
    }
    const int npix = (int)(n_tiles * 64);
    int end_bit = key_bits;
    while ((1ull << (end_bit - key_bits)) <= (uint64_t)P) end_bit++;
    // workspace
    size_t tmp_sort = 0, tmp_red = 0;
    hipcub::DoubleBuffer<uint32_t> dk(nullptr, nullptr), dv(nullptr, nullptr);
    TILER_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, dk, dv, npix, 0, end_bit, stream));
    hipcub::TransformInputIterator<Dl3Sum, Dl3Expand, const uint32_t *> it_in(nullptr, Dl3Expand());
    TILER_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(nullptr, tmp_red, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                      it_in, (Dl3Sum *)nullptr, (int *)nullptr, Dl3SumOp(), npix,
                                                      stream));
    const size_t np = (size_t)std::max(npix, 1);
    const size_t b_keys = 4 * np, b_sum = sizeof(Dl3Sum) * np, b_tmp = std::max(tmp_sort, tmp_red) + 256;
    const size_t b_pairs = 4 * ((size_t)P + 2), b_table = 2 * b_keys + 8 * 1024;  // + slack for unclamped loads
    // The workspace is the sum of the carved pieces, each rounded up to 256 bytes (the same rounding as take()).
    const size_t sizes[] = {b_keys, b_keys, b_keys, b_keys, b_keys, b_sum, b_tmp, b_pairs, b_pairs, b_pairs,
                            b_table, b_table, 4 * b_keys, 4 * (size_t)P * palsize};
    size_t bytes = 0;
    for (size_t b : sizes) bytes += (b + 255) & ~(size_t)255;
    char *ws = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&ws, bytes));
    char *cur = ws;
    auto take = [&](size_t b) {
        char *r = cur;
        cur += (b + 255) & ~(size_t)255;
        return r;
    };
    uint32_t *k0 = (uint32_t *)take(b_keys), *k1 = (uint32_t *)take(b_keys);
    uint32_t *v0 = (uint32_t *)take(b_keys), *v1 = (uint32_t *)take(b_keys);
    uint32_t *ukeys = (uint32_t *)take(b_keys);
    Dl3Sum *agg = (Dl3Sum *)take(b_sum);
    void *tmp = take(b_tmp);
    int *d_nruns = (int *)take(b_pairs);
    int *d_seg = (int *)take(b_pairs);
    int *d_uc = (int *)take(b_pairs);
    Dl3Tab t;
    t.QN = (uint2 *)take(b_table);  // scans
    t.EC = (uint2 *)take(b_table);  // pass 1
    t.V = (uint4 *)take(4 * b_keys);
    int *d_list = (int *)k0;  // the sort buffers are free once the table exists
    int32_t *d_pal = (int32_t *)take(4 * (size_t)P * palsize);
    if ((size_t)(cur - ws) != bytes) {
        hipFree(ws);
        set_error("quantize_palettes: workspace layout mismatch");
        return -1;
    }
    int rc = -1, step = 0;  // step: the failing call (error message)
    std::vector<int> seg(P + 1);
    do {
        if (hipMemsetAsync(d_uc, 0, 4 * (P + 2), stream) != hipSuccess) { step = 1; break; }
        if (hipMemsetAsync(d_nruns, 0, 4, stream) != hipSuccess) { step = 2; break; }
        if (npix > 0) {
            KTimer tk("dl3_table", stream);
            hipLaunchKernelGGL(dl3_keys_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, stream, d_rgb, d_pal_of,
                               d_active, n_tiles, P, bpc, k0, v0, d_uc);
            if (hipGetLastError() != hipSuccess) { step = 3; break; }
            hipcub::DoubleBuffer<uint32_t> kb(k0, k1), vb(v0, v1);
            size_t ts = tmp_sort;
            if (hipcub::DeviceRadixSort::SortPairs(tmp, ts, kb, vb, npix, 0, end_bit, stream) != hipSuccess) { step = 4; break; }
            hipcub::TransformInputIterator<Dl3Sum, Dl3Expand, const uint32_t *> vin(vb.Current(), Dl3Expand());
            size_t tr = tmp_red;
            if (hipcub::DeviceReduce::ReduceByKey(tmp, tr, (const uint32_t *)kb.Current(), ukeys, vin, agg, d_nruns,
                                                  Dl3SumOp(), npix, stream) != hipSuccess) {
                step = 14;
                break;
            }
        }
        hipLaunchKernelGGL(dl3_seg_kernel, dim3((P + 256) / 256), dim3(256), 0, stream, ukeys, d_nruns, P, bpc, d_seg);
        if (hipGetLastError() != hipSuccess) { step = 5; break; }
        if (hipMemcpyAsync(seg.data(), d_seg, 4 * (P + 1), hipMemcpyDeviceToHost, stream) != hipSuccess) { step = 6; break; }
        if (hipMemcpyAsync(use_count, d_uc, 4 * P, hipMemcpyDeviceToHost, stream) != hipSuccess) { step = 7; break; }
        if (hipStreamSynchronize(stream) != hipSuccess) { step = 8; break; }
        const int total = seg[P];
        if (total > 0) {
            hipLaunchKernelGGL(dl3_init_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, agg, d_seg, P,
                               t);
            if (hipGetLastError() != hipSuccess) { step = 9; break; }
        }
        {
            KTimer tp("dl3_pass1", stream);
            if (total > 0)
                hipLaunchKernelGGL(dl3_pass1_kernel, dim3((unsigned)std::min(65536, (total + 3) / 4)), dim3(256), 0, stream,
                                   ukeys, d_seg, P, bpc, t);
            if (hipGetLastError() != hipSuccess) { step = 10; break; }
        }
        {
            KTimer tr("dl3_reduce", stream);
            Dl3Args ra;
            ra.t = t;
            ra.seg = d_seg;
            ra.quant_to = palsize;
            ra.list = d_list;
            ra.lcap = std::max(1, std::min(DL3_LCAP, g_dl3_lcap.load()));
            ra.pal = d_pal;
            hipLaunchKernelGGL(dl3_reduce_kernel, dim3(P), dim3(DL3_T), 0, stream, ra);
            if (hipGetLastError() != hipSuccess) { step = 11; break; }
        }
        if (hipMemcpyAsync(pal_out, d_pal, 4 * (size_t)P * palsize, hipMemcpyDeviceToHost, stream) != hipSuccess) { step = 12; break; }
        if (hipStreamSynchronize(stream) != hipSuccess) { step = 13; break; }
        for (int p = 0; p < P; p++) {
            if (hist) hist[p] = seg[p + 1] - seg[p];
            sort_palette_cmulhs(pal_out + (size_t)p * palsize, palsize);  // CMPal.Sort (main.pas:2413)
        }
        rc = 0;
    } while (0);
    if (rc) {
        const hipError_t e = hipGetLastError();
        set_error("quantize_palettes: HIP failure at step " + std::to_string(step) + " (" + hipGetErrorString(e) +
                  "), " + std::to_string(npix) + " pixels, " + std::to_string(P) + " pairs");
    }
    (void)hipFree(ws);
    return rc;
}

int quantize_palettes_host(long n_tiles, const int32_t *rgb, const int32_t *pal_of, const uint8_t *active, int P,
                           int palsize, int bpc, int32_t *pal_out, int32_t *use_count, int32_t *hist) {
    if (n_tiles < 0 || (n_tiles > 0 && (!rgb || !pal_of))) {
        set_error("quantize_palettes: invalid arguments");
        return -1;
    }
    const size_t b_rgb = (size_t)n_tiles * 256, b_po = (size_t)n_tiles * 4, b_act = active ? (size_t)n_tiles : 0;
    char *buf = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&buf, b_rgb + b_po + b_act + 64));
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        (void)hipFree(buf);
        set_error("quantize_palettes: stream creation failed");
        return -1;
    }
    int rc = -1;
    do {
        if (hipMemcpyAsync(buf, rgb, b_rgb, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(buf + b_rgb, pal_of, b_po, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (active && hipMemcpyAsync(buf + b_rgb + b_po, active, b_act, hipMemcpyHostToDevice, st) != hipSuccess) break;
        rc = quantize_palettes_dev(n_tiles, (const int32_t *)buf, (const int32_t *)(buf + b_rgb),
                                   active ? (const uint8_t *)(buf + b_rgb + b_po) : nullptr, P, palsize, bpc, pal_out,
                                   use_count, hist, st);
    } while (0);
    if (rc && !last_error()[0]) set_error("quantize_palettes: HIP copy failed");
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    (void)hipFree(buf);
    return rc;
}

}  // namespace tiler

// kdtree.hip -- ANN 1.1.2 kd-tree (ANN_KD_STD) build over an HBM dataset + the pruning check / exact replay
// that make the MFMA search return ANN's own answer among equal distances (kdtree.hpp).
//
// Build, level by level (every node of a level at once), entirely on the device (the shape is implicit, so the host
// plans every level before any data exists; nothing comes back until the tree is done):
//   big nodes (> KD_CH points): kd_spread_big_kernel, one wave per KD_CH-point chunk, per-dimension min / max
//                      (annSpread) folded into the node with order-preserving integer atomics; kd_select_big_kernel
//                      picks cut_dim = first maximum of max - min (fp32, annMaxSpread); kd_gather_kernel writes
//                      the node's cut-dimension keys in pidx order, one wave per chunk
//   small nodes:       kd_small_kernel, one wave per node does all three
//   kd_median_big_kernel: annMedianSplit's quickselect on each node's (key, index) pairs by a workgroup, bit for bit
//                      (Hoare's partition ranked in parallel): the permutation it leaves decides which of several equal
//                      keys go LO, and so the rest of the tree
//   subtrees of <= KD_SUB points: kd_subtree_waves_kernel, one workgroup each; then the cell bounds and positions
#include <float.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <vector>

#include "kdorder_dev.hpp"
#include "kdtree.hpp"

namespace tiler {

static constexpr int KD_CH = 128;  // points per spread chunk (one wave) of a big node

struct KdChunk {
    int node, s, e;  // big-node index, positions [s, e)
};

struct KdNodeDev {
    int s, e;
};

// order-preserving float <-> uint32 (min / max of the encodings = encodings of the min / max)
__device__ __forceinline__ unsigned f2o(float f) {
    const unsigned b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float o2f(unsigned o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o); }

// min / max of pidx[s..e) along dims d0 + lane + 64 j (j < 4), rows read 4 at a time (independent loads)
__device__ __forceinline__ void kd_minmax(const float *__restrict__ rows, int dd, const int *__restrict__ pidx, int s,
                                          int e, int d0, float (&mn)[4], float (&mx)[4]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        mn[j] = INFINITY;
        mx[j] = -INFINITY;
    }
    int i = s;
    for (; i + 4 <= e; i += 4) {
        const float *r[4];
#pragma unroll
        for (int u = 0; u < 4; u++) r[u] = rows + (long)pidx[i + u] * dd;
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int d = d0 + j * 64 + lane;
                v[u][j] = d < dd ? r[u][d] : 0.0f;
            }
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                mn[j] = fminf(mn[j], v[u][j]);
                mx[j] = fmaxf(mx[j], v[u][j]);
            }
    }
    for (; i < e; i++) {
        const float *r = rows + (long)pidx[i] * dd;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = d0 + j * 64 + lane;
            const float v = d < dd ? r[d] : 0.0f;
            mn[j] = fminf(mn[j], v);
            mx[j] = fmaxf(mx[j], v);
        }
    }
}

// wave argmax of (spread, -dim): annMaxSpread's first maximum; an all-zero spread picks dimension 0
__device__ __forceinline__ int kd_first_max(float best, int bd) {
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int od = __shfl_xor(bd, o, 64);
        if (ob > best || (ob == best && od < bd)) {
            best = ob;
            bd = od;
        }
    }
    return best > 0.0f ? bd : 0;
}

__global__ __launch_bounds__(256) void kd_spread_big_kernel(const float *__restrict__ rows, int dd,
                                                            const int *__restrict__ pidx,
                                                            const KdChunk *__restrict__ ch, int nch,
                                                            unsigned *__restrict__ omin, unsigned *__restrict__ omax) {
    // one wave per chunk; the waves of a workgroup that share a node fold their minima / maxima in LDS first, so each
    // node dimension takes one pair of atomics per workgroup run of its chunks, not one per chunk
    __shared__ float smn[4][256], smx[4][256];
    __shared__ int snode[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 4 + w;
    const bool valid = c < nch;
    const KdChunk k = valid ? ch[c] : KdChunk{-1, 0, 0};
    if (lane == 0) snode[w] = k.node;
    for (int d0 = 0; d0 < dd; d0 += 256) {
        float mn[4], mx[4];
        kd_minmax(rows, dd, pidx, k.s, k.e, d0, mn, mx);  // an invalid wave's empty range: +inf / -inf
#pragma unroll
        for (int j = 0; j < 4; j++) {
            smn[w][j * 64 + lane] = mn[j];
            smx[w][j * 64 + lane] = mx[j];
        }
        __syncthreads();
        if (valid && (w == 0 || snode[w - 1] != k.node)) {  // the first wave of its node's run in this workgroup
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int d = d0 + j * 64 + lane;
                float a = smn[w][j * 64 + lane], b = smx[w][j * 64 + lane];
                for (int u = w + 1; u < 4 && snode[u] == k.node; u++) {
                    a = fminf(a, smn[u][j * 64 + lane]);
                    b = fmaxf(b, smx[u][j * 64 + lane]);
                }
                if (d < dd) {
                    atomicMin(&omin[(long)k.node * dd + d], f2o(a));
                    atomicMax(&omax[(long)k.node * dd + d], f2o(b));
                }
            }
        }
        __syncthreads();
    }
}

// one wave per big node: the cut dimension (also the root box when box != null)
__global__ __launch_bounds__(256) void kd_select_big_kernel(int dd, int nbig, const unsigned *__restrict__ omin,
                                                            const unsigned *__restrict__ omax, int *__restrict__ cut_dim,
                                                            float *__restrict__ box) {
    const int lane = threadIdx.x & 63;
    const int nd = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nd >= nbig) return;
    float best = -INFINITY;
    int bd = 0x7fffffff;
    for (int d = lane; d < dd; d += 64) {
        const float mn = o2f(omin[(long)nd * dd + d]), mx = o2f(omax[(long)nd * dd + d]);
        if (box) {  // the root node: annEnclRect
            box[d] = mn;
            box[dd + d] = mx;
        }
        const float spr = mx - mn;
        if (spr > best) {  // lane-local dims ascend: the first maximum
            best = spr;
            bd = d;
        }
    }
    const int cd = kd_first_max(best, bd);
    if (lane == 0) cut_dim[nd] = cd;
}

// keys[i] = rows[pidx[i]][cut_dim of the chunk's node], one wave per chunk
__global__ __launch_bounds__(256) void kd_gather_kernel(const float *__restrict__ rows, int dd,
                                                        const int *__restrict__ pidx, const KdChunk *__restrict__ ch,
                                                        int nch, const int *__restrict__ cut_dim,
                                                        float *__restrict__ keys) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch) return;
    const KdChunk k = ch[c];
    const int cd = cut_dim[k.node];
    for (int i = k.s + lane; i < k.e; i += 64) keys[i] = rows[(long)pidx[i] * dd + cd];
}

// one wave per small node: spread, cut dimension and keys in one pass
__global__ __launch_bounds__(256) void kd_small_kernel(const float *__restrict__ rows, int dd,
                                                       const int *__restrict__ pidx,
                                                       const KdNodeDev *__restrict__ nodes, int nn,
                                                       int *__restrict__ cut_dim, float *__restrict__ keys,
                                                       float *__restrict__ box) {
    const int lane = threadIdx.x & 63;
    const int nd = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nd >= nn) return;
    const KdNodeDev N = nodes[nd];
    float best = -INFINITY;
    int bd = 0x7fffffff;
    for (int d0 = 0; d0 < dd; d0 += 256) {
        float mn[4], mx[4];
        kd_minmax(rows, dd, pidx, N.s, N.e, d0, mn, mx);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = d0 + j * 64 + lane;
            if (d < dd) {
                if (box) {
                    box[d] = mn[j];
                    box[dd + d] = mx[j];
                }
                const float spr = mx[j] - mn[j];
                if (spr > best || (spr == best && d < bd)) {
                    best = spr;
                    bd = d;
                }
            }
        }
    }
    const int cd = kd_first_max(best, bd);
    if (lane == 0) cut_dim[nd] = cd;
    for (int i = N.s + lane; i < N.e; i += 64) keys[i] = rows[(long)pidx[i] * dd + cd];
}

// annMedianSplit (kd_util.cpp) on one big node's (key, index) pairs, key[i] = PA(i, cut_dim), by a whole workgroup
// (round 3; until then a host thread ran it per node, with the keys round-tripped every level).  Sequentially:
//     l = 0, r = n-1; while l < r: i = (l+r)/2; if key[i] > key[r] swap(i, r); swap(l, i); c = key[l];
//       i = l, k = r; loop { while key[++i] < c; while key[--k] > c; if i < k swap(i, k) else break }; swap(l, k);
//       k > n_lo -> r = k-1, k < n_lo -> l = k+1, else stop
//     then the first maximum of key[0..n_lo) swapped to n_lo - 1; cut_val = (key[n_lo-1] + key[n_lo]) / 2.
// Hoare's partition is data-parallel.  With the pivot c, the i-scan stops at the "left stoppers" of the ORIGINAL
// array (p in (l, r] with key[p] >= c, ascending L_1 < L_2 < ...; key[r] >= c ends it) and the k-scan at the "right
// stoppers" (p in [l, r) with key[p] <= c, descending R_1 > R_2 > ...; key[l] = c ends it): positions the scans
// still have to cross are untouched by earlier swaps, and a swapped position stops the scan that reaches it next,
// exactly at the point where the loop then ends.  So the loop swaps the pairs (L_j, R_j) with L_j < R_j -- a prefix
// j < J, since L ascends and R descends -- and stops with k = R_J (J = 1) or max(R_J, L_{J-1}).  L_j < R_j iff the
// number of right stoppers above L_j is >= j, which each lane decides from the ranks alone.  Per iteration: each wave
// ranks a contiguous segment by ballots (two passes), writes the stoppers' positions by rank, the J-1 swaps run in
// parallel (their positions are distinct), then swap(l, k).  Same comparisons, same permutation, same cut value.
static constexpr int KD_MW = 16;    // waves per big-node workgroup
static constexpr int KD_TAIL = 2048;  // a range this short finishes in LDS by one wave (kd_qselect_wave)
__device__ __forceinline__ void kd_swap(float *kk, int *ii, int a, int b) {
    const float tk = kk[a];
    kk[a] = kk[b];
    kk[b] = tk;
    const int ti = ii[a];
    ii[a] = ii[b];
    ii[b] = ti;
}

__device__ __forceinline__ void kd_wsync() {  // a wave's LDS writes visible to its other lanes
    __builtin_amdgcn_s_waitcnt(0xc07f);         // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// annMedianSplit's loop from the state (l, r) with n_lo in [l, r] (the loop's invariant), by one wave
__device__ __forceinline__ void kd_qselect_wave(float *kk, int *ii, int l, int r, int n_lo, int *Lp, int *Rp) {
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    while (l < r) {  // l, r, k: wave-uniform
        if (lane == 0) {
            const int i = (r + l) / 2;
            if (kk[i] > kk[r]) kd_swap(kk, ii, i, r);
            kd_swap(kk, ii, l, i);
        }
        kd_wsync();
        const float c = kk[l];
        int tot_r = 0;
        for (int p0 = l; p0 <= r; p0 += 64) {
            const int p = p0 + lane;
            const float v = p <= r ? kk[p] : 0.0f;
            tot_r += __popcll(__ballot(p < r && !(v > c)));
        }
        int bl = 0, br = 0, np = 0;
        for (int p0 = l; p0 <= r; p0 += 64) {
            const int p = p0 + lane;
            const float v = p <= r ? kk[p] : 0.0f;
            // stoppers where the scans' loop tests fail (NaN keys stop both scans, as the sequential comparisons do)
            const bool isl = p <= r && p > l && !(v < c), isr = p < r && !(v > c);
            const unsigned long long bL = __ballot(isl), bR = __ballot(isr);
            const int jl = bl + __popcll(bL & below) + 1;  // rank from the left (1-based)
            const int rb = br + __popcll(bR & below);      // right stoppers below p
            if (isl) Lp[jl - 1] = p;
            if (isr) Rp[tot_r - rb - 1] = p;
            if (isl && tot_r - rb - (isr ? 1 : 0) >= jl) np++;  // R_jl > p: pair jl is swapped
            bl += __popcll(bL);
            br += __popcll(bR);
        }
        for (int o = 32; o > 0; o >>= 1) np += __shfl_xor(np, o, 64);
        kd_wsync();
        for (int j = lane; j < np; j += 64) kd_swap(kk, ii, Lp[j], Rp[j]);
        kd_wsync();
        int k = Rp[np];
        if (np > 0) k = max(k, Lp[np - 1]);
        if (lane == 0) kd_swap(kk, ii, l, k);
        kd_wsync();
        if (k > n_lo)
            r = k - 1;
        else if (k < n_lo)
            l = k + 1;
        else
            break;
    }
}

__global__ __launch_bounds__(64 * KD_MW) void kd_median_big_kernel(float *__restrict__ keys, int *__restrict__ pidx,
                                                                   const KdNodeDev *__restrict__ nodes,
                                                                   const int *__restrict__ cut_dim,
                                                                   int *__restrict__ lpos, int *__restrict__ rpos,
                                                                   int *__restrict__ cd_out, float *__restrict__ cv_out) {
    __shared__ int s_l, s_r;
    __shared__ float s_c;
    __shared__ int wl[KD_MW], wr[KD_MW], wp[KD_MW];
    __shared__ float wv[KD_MW];
    __shared__ float t_k[KD_TAIL];
    __shared__ int t_i[KD_TAIL], t_l[KD_TAIL], t_r[KD_TAIL];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const KdNodeDev N = nodes[blockIdx.x];
    float *kk = keys + N.s;
    int *ii = pidx + N.s, *Lp = lpos + N.s, *Rp = rpos + N.s;
    const int n = N.e - N.s, n_lo = n / 2;
    const unsigned long long below = (1ull << lane) - 1ull;
    if (tid == 0) {
        s_l = 0;
        s_r = n - 1;
    }
    __syncthreads();
    for (;;) {
        const int l = s_l, r = s_r;  // uniform: read after the barrier
        if (l >= r) break;
        if (r - l < KD_TAIL) {  // the rest of the loop on an LDS copy of [l, r] by one wave (no global round trips)
            for (int p = l + tid; p <= r; p += 64 * KD_MW) {
                t_k[p - l] = kk[p];
                t_i[p - l] = ii[p];
            }
            __syncthreads();
            if (w == 0) kd_qselect_wave(t_k, t_i, 0, r - l, n_lo - l, t_l, t_r);
            __syncthreads();
            for (int p = l + tid; p <= r; p += 64 * KD_MW) {
                kk[p] = t_k[p - l];
                ii[p] = t_i[p - l];
            }
            __syncthreads();
            break;
        }
        if (tid == 0) {
            const int i = (r + l) / 2;
            if (kk[i] > kk[r]) kd_swap(kk, ii, i, r);
            kd_swap(kk, ii, l, i);
            s_c = kk[l];
        }
        __syncthreads();
        const float c = s_c;
        const int seg = (r - l + KD_MW) / KD_MW;  // ceil((r - l + 1) / KD_MW)
        const int a0 = l + w * seg, a1 = min(r + 1, a0 + seg);
        int nl = 0, nr = 0;
        for (int p0 = a0; p0 < a1; p0 += 256) {  // 4 loads in flight per lane before their ballots
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = p0 + 64 * u + lane;
                v[u] = p < a1 ? kk[p] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = p0 + 64 * u + lane;
                nl += __popcll(__ballot(p < a1 && p > l && !(v[u] < c)));
                nr += __popcll(__ballot(p < a1 && p < r && !(v[u] > c)));
            }
        }
        if (lane == 0) {
            wl[w] = nl;
            wr[w] = nr;
        }
        __syncthreads();
        int bl = 0, br = 0, tot_r = 0;
        for (int x = 0; x < KD_MW; x++) {
            if (x < w) {
                bl += wl[x];
                br += wr[x];
            }
            tot_r += wr[x];
        }
        int np = 0;
        for (int p0 = a0; p0 < a1; p0 += 256) {  // 4 loads in flight, then the 4 pieces in position order
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = p0 + 64 * u + lane;
                v[u] = p < a1 ? kk[p] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = p0 + 64 * u + lane;
                // a stopper is where the scan's loop test FAILS: !(key < c) / !(key > c), so a NaN key (or a NaN
                // pivot) stops both scans exactly as the sequential loop's comparisons do (and position l always
                // stops the k-scan)
                const bool isl = p < a1 && p > l && !(v[u] < c), isr = p < a1 && p < r && !(v[u] > c);
                const unsigned long long bL = __ballot(isl), bR = __ballot(isr);
                const int jl = bl + __popcll(bL & below) + 1;  // rank from the left (1-based)
                const int rb = br + __popcll(bR & below);      // right stoppers below p
                if (isl) Lp[jl - 1] = p;
                if (isr) Rp[tot_r - rb - 1] = p;  // rank from the right: tot_r - rb
                if (isl && tot_r - rb - (isr ? 1 : 0) >= jl) np++;  // R_jl > p: pair jl is swapped
                bl += __popcll(bL);
                br += __popcll(bR);
            }
        }
        for (int o = 32; o > 0; o >>= 1) np += __shfl_xor(np, o, 64);
        if (lane == 0) wp[w] = np;
        __syncthreads();
        np = 0;
        for (int x = 0; x < KD_MW; x++) np += wp[x];
        for (int j = tid; j < np; j += 64 * KD_MW) kd_swap(kk, ii, Lp[j], Rp[j]);
        __syncthreads();
        if (tid == 0) {
            int k = Rp[np];  // R_J, J = np + 1 (<= tot_r: position l is the last right stopper, never paired)
            if (np > 0) k = max(k, Lp[np - 1]);
            kd_swap(kk, ii, l, k);
            if (k > n_lo)
                s_r = k - 1;
            else if (k < n_lo)
                s_l = k + 1;
            else
                s_l = s_r = k;
        }
        __syncthreads();
    }
    // the first maximum of kk[0..n_lo) to n_lo - 1.  Sequentially m = 0, then m = i where key[i] > key[m]: a NaN key
    // never replaces m, and a NaN key[0] is never replaced -- so NaN keys are skipped here and key[0] = NaN decides
    // below
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < n_lo; i += 64 * KD_MW) {
        const float v = kk[i];
        if (v == v && (v > bv || bi == 0x7fffffff)) {  // a thread's indices ascend: strict > keeps its first
            bv = v;
            bi = i;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (oi != 0x7fffffff && (bi == 0x7fffffff || ov > bv || (ov == bv && oi < bi))) {
            bv = ov;
            bi = oi;
        }
    }
    if (lane == 0) {
        wv[w] = bv;
        wp[w] = bi;
    }
    __syncthreads();
    if (tid == 0) {
        int k = 0x7fffffff;
        float c = -INFINITY;
        for (int x = 0; x < KD_MW; x++)
            if (wp[x] != 0x7fffffff && (k == 0x7fffffff || wv[x] > c || (wv[x] == c && wp[x] < k))) {
                c = wv[x];
                k = wp[x];
            }
        if (n_lo > 0 && (k == 0x7fffffff || kk[0] != kk[0])) k = 0;  // key[0] NaN (or every key NaN): m stays 0
        if (n_lo > 0) kd_swap(kk, ii, n_lo - 1, k);
        const int m = N.s + n_lo;
        cd_out[m] = cut_dim[blockIdx.x];
        cv_out[m] = (float)(((double)(kk[n_lo - 1] + kk[n_lo])) / 2.0);
    }
}

// ANNkd_split::cd_bnds of every internal node (rkd_tree: the LO child descends with bnd_box.hi[cd] = cv, the HI child
// with .lo[cd] = cv; the node records lo[cd] / hi[cd] on entry): one thread per position p, two root walks -- find
// the node split at p and its cut dimension, then apply the ancestors cutting that dimension, root first.
__global__ __launch_bounds__(256) void kd_bounds_kernel(int n, int bs, const int *__restrict__ cd,
                                                        const float *__restrict__ cv, const float *__restrict__ box,
                                                        int dd, float *__restrict__ lo_out, float *__restrict__ hi_out) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    int s = 0, e = n;
    bool found = false;
    while (e - s > bs) {
        const int m = s + (e - s) / 2;
        if (p == m) {
            found = true;
            break;
        }
        if (p < m)
            e = m;
        else
            s = m;
    }
    if (!found) return;
    const int c = cd[p];
    float lo = box[c], hi = box[dd + c];
    s = 0;
    e = n;
    for (;;) {
        const int m = s + (e - s) / 2;
        if (m == p) break;
        const bool same = cd[m] == c;
        if (p < m) {
            if (same) hi = cv[m];
            e = m;
        } else {
            if (same) lo = cv[m];
            s = m;
        }
    }
    lo_out[p] = lo;
    hi_out[p] = hi;
}

__global__ __launch_bounds__(256) void kd_pos_kernel(int n, const int *__restrict__ pidx, int *__restrict__ pos) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) pos[pidx ? pidx[i] : i] = i;  // pidx null: the identity (SkeletonTree's pidx[i] = i)
}

// A whole subtree of <= KD_SUB points per workgroup, entirely on the device: every node's annSpread / annMaxSpread
// cut dimension, its keys into LDS and annMedianSplit's quickselect on the LDS copy -- the same comparisons, swaps and
// cut value as kd_median_big_kernel -- so the subtree's permutation, cut dimensions and cut values are ANN's.  Nodes of
// one level own disjoint ranges of key / idx and distinct output slots, so they run concurrently.
//   * a level of >= KD_SW nodes: one wave per node (lanes over dimensions, a wave reduction for the first maximum);
//   * a level of fewer nodes (the subtree's top levels, where one wave per node left most of the workgroup idle):
//     KD_SW / nn waves per node, each folding every (KD_SW / nn)-th point into per-wave minima / maxima in LDS;
//   * the quickselect by the node's wave: Hoare's partition ranked by ballots (kd_median_big_kernel's scheme at wave
//     scale) instead of one lane walking the keys.
static constexpr int KD_SUB = 1024;
static constexpr int KD_SW = 16;
static constexpr int KD_PD = 256;  // dimensions of the multi-wave partials (larger dd: one wave per node)
static constexpr int KD_DFS = 32;  // nodes this small are finished depth first by one wave (stack depth <= 6 + 1)

// min / max over points idx[s], idx[s + step], ... (< e) along dims d0 + lane + 64 j (j < 4); 4 points per round
__device__ __forceinline__ void kd_minmax_idx(const float *__restrict__ rows, int dd, const int *idx, int s, int e,
                                              int step, int d0, float (&mn)[4], float (&mx)[4]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        mn[j] = INFINITY;
        mx[j] = -INFINITY;
    }
    int i = s;
    for (; i + 3 * step < e; i += 4 * step) {
        const float *r[4];
#pragma unroll
        for (int u = 0; u < 4; u++) r[u] = rows + (long)idx[i + u * step] * dd;
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int d = d0 + j * 64 + lane;
                v[u][j] = d < dd ? r[u][d] : 0.0f;
            }
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                mn[j] = fminf(mn[j], v[u][j]);
                mx[j] = fmaxf(mx[j], v[u][j]);
            }
    }
    for (; i < e; i += step) {
        const float *r = rows + (long)idx[i] * dd;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = d0 + j * 64 + lane;
            const float v = d < dd ? r[d] : 0.0f;
            mn[j] = fminf(mn[j], v);
            mx[j] = fmaxf(mx[j], v);
        }
    }
}

// annMedianSplit on kk[0..n) / ii[0..n) (LDS) by one wave; Lp / Rp: n ints of LDS scratch.  Leaves the keys and
// indices permuted exactly as the sequential quickselect does (kd_median_big_kernel's derivation), the first maximum
// of kk[0..n_lo) swapped to n_lo - 1.
__device__ __forceinline__ void kd_median_wave(float *kk, int *ii, int n, int *Lp, int *Rp) {
    const int lane = threadIdx.x & 63;
    const int n_lo = n / 2;
    kd_qselect_wave(kk, ii, 0, n - 1, n_lo, Lp, Rp);
    // the first maximum of kk[0..n_lo) to n_lo - 1 (NaN keys as in kd_median_big_kernel)
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = lane; i < n_lo; i += 64) {
        const float v = kk[i];
        if (v == v && (v > bv || bi == 0x7fffffff)) {
            bv = v;
            bi = i;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (oi != 0x7fffffff && (bi == 0x7fffffff || ov > bv || (ov == bv && oi < bi))) {
            bv = ov;
            bi = oi;
        }
    }
    if (n_lo > 0 && (bi == 0x7fffffff || kk[0] != kk[0])) bi = 0;
    if (n_lo > 0 && lane == 0) kd_swap(kk, ii, n_lo - 1, bi);
    kd_wsync();
}

__global__ __launch_bounds__(64 * KD_SW) void kd_subtree_waves_kernel(const float *__restrict__ rows, int dd,
                                                                     int *__restrict__ pidx,
                                                                     const KdNodeDev *__restrict__ roots, int bs,
                                                                     int *__restrict__ cd_out, float *__restrict__ cv_out) {
    __shared__ float key[KD_SUB];
    __shared__ int idx[KD_SUB];
    __shared__ int lpos[KD_SUB], rpos[KD_SUB];
    __shared__ int2 lvl[2][KD_SUB / 2 + 1];
    __shared__ int nlvl[2];
    __shared__ float pmn[KD_SW][KD_PD], pmx[KD_SW][KD_PD];
    __shared__ int gcd[KD_SW];
    __shared__ int2 stk[KD_SW][16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const KdNodeDev R = roots[blockIdx.x];
    const int S = R.s, m_all = R.e - R.s;
    for (int i = tid; i < m_all; i += 64 * KD_SW) idx[i] = pidx[S + i];
    if (tid == 0) {
        lvl[0][0] = make_int2(0, m_all);
        nlvl[0] = 1;  // the root is processed even when it is a leaf (as the round-1 kernel did; its cut is never read)
        nlvl[1] = 0;
    }
    __syncthreads();
    // a node's cut dimension known: keys gathered, median, outputs, children (one wave; keys already in LDS)
    // children of <= KD_DFS points go on the wave's own stack and are finished by that wave, depth first, without the
    // level barriers (the deep levels are many tiny nodes whose cost is fixed latency)
    int top = 0;  // wave-uniform depth of this wave's stack
    auto split_node = [&](int s, int e, int cd, int nxt) __attribute__((always_inline)) {
        const int n = e - s, n_lo = n / 2;
        kd_median_wave(key + s, idx + s, n, lpos + s, rpos + s);
        const int m = s + n_lo;
        if (lane == 0) {
            const float *kk = key + s;
            cd_out[S + m] = cd;
            cv_out[S + m] = (float)(((double)(kk[n_lo > 0 ? n_lo - 1 : 0] + kk[n_lo])) / 2.0);
        }
        if (e - m > bs) {
            if (e - m > KD_DFS) {
                if (lane == 0) lvl[nxt][atomicAdd(&nlvl[nxt], 1)] = make_int2(m, e);
            } else {
                if (lane == 0) stk[w][top] = make_int2(m, e);
                top++;
            }
        }
        if (m - s > bs) {
            if (m - s > KD_DFS) {
                if (lane == 0) lvl[nxt][atomicAdd(&nlvl[nxt], 1)] = make_int2(s, m);
            } else {
                if (lane == 0) stk[w][top] = make_int2(s, m);
                top++;
            }
        }
    };
    // one node by one wave: annSpread / annMaxSpread over its points, keys to LDS, median, children
    auto wave_node = [&](int s, int e, int nxt) __attribute__((always_inline)) {
        float best = -INFINITY;
        int bd = 0x7fffffff;
        for (int d0 = 0; d0 < dd; d0 += 256) {
            float mn[4], mx[4];
            kd_minmax_idx(rows, dd, idx, s, e, 1, d0, mn, mx);
#pragma unroll
            for (int q = 0; q < 4; q++) {  // this lane's dimensions ascend: strict > keeps the first
                const int d = d0 + q * 64 + lane;
                const float spr = mx[q] - mn[q];
                if (d < dd && spr > best) {
                    best = spr;
                    bd = d;
                }
            }
        }
        const int cd = kd_first_max(best, bd);
        for (int i = s + lane; i < e; i += 64) key[i] = rows[(long)idx[i] * dd + cd];
        kd_wsync();
        split_node(s, e, cd, nxt);
    };
    auto drain_stack = [&](int nxt) __attribute__((always_inline)) {
        while (top > 0) {
            kd_wsync();
            const int2 nd = stk[w][--top];
            wave_node(nd.x, nd.y, nxt);
        }
    };
    for (int L = 0;; L++) {
        const int cur = L & 1, nxt = cur ^ 1;
        const int nn = nlvl[cur];
        if (nn == 0) break;  // uniform: read after the barrier
        if (nn < KD_SW && dd <= KD_PD) {
            const int gw = KD_SW / nn, j = w / gw, sub = w - j * gw;
            int s = 0, e = 0;
            if (j < nn) {
                const int2 nd = lvl[cur][j];
                s = nd.x;
                e = nd.y;
                for (int d0 = 0; d0 < dd; d0 += 256) {
                    float mn[4], mx[4];
                    kd_minmax_idx(rows, dd, idx, s + sub, e, gw, d0, mn, mx);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int d = d0 + q * 64 + lane;
                        if (d < dd) {
                            pmn[w][d] = mn[q];
                            pmx[w][d] = mx[q];
                        }
                    }
                }
            }
            __syncthreads();
            if (j < nn && sub == 0) {
                float best = -INFINITY;
                int bd = 0x7fffffff;
                for (int d = lane; d < dd; d += 64) {  // this lane's dimensions ascend: strict > keeps the first
                    float mn = pmn[w][d], mx = pmx[w][d];
                    for (int g = 1; g < gw; g++) {
                        mn = fminf(mn, pmn[w + g][d]);
                        mx = fmaxf(mx, pmx[w + g][d]);
                    }
                    const float spr = mx - mn;
                    if (spr > best) {
                        best = spr;
                        bd = d;
                    }
                }
                const int cd = kd_first_max(best, bd);
                if (lane == 0) gcd[j] = cd;
            }
            __syncthreads();
            if (j < nn) {
                const int cd = gcd[j];
                for (int i = s + sub * 64 + lane; i < e; i += gw * 64) key[i] = rows[(long)idx[i] * dd + cd];
            }
            __syncthreads();
            if (j < nn && sub == 0) {
                split_node(s, e, gcd[j], nxt);
                drain_stack(nxt);
            }
        } else {
            for (int j = w; j < nn; j += KD_SW) {
                const int2 nd = lvl[cur][j];
                wave_node(nd.x, nd.y, nxt);
                drain_stack(nxt);
            }
        }
        __syncthreads();
        if (tid == 0) nlvl[cur] = 0;
        __syncthreads();
    }
    for (int i = tid; i < m_all; i += 64 * KD_SW) pidx[S + i] = idx[i];
}

KdOrder KdTree::view() const {
    KdOrder o;
    o.pos = d_pos;
    o.pidx = d_pidx;
    o.cd = d_cd;
    o.cv = d_cv;
    o.lo = d_lo;
    o.hi = d_hi;
    o.box_lo = d_box;
    o.box_hi = d_box ? d_box + dd : nullptr;
    o.n = n;
    o.bs = bs;
    o.dd = dd;
    return o;
}

void kd_tree_destroy(KdTree *t, bool synced) {
    if (!t) return;
    if (!synced) (void)hipDeviceSynchronize();  // dfree files the blocks for reuse: nothing may still read them (hipFree's rule)
    dfree(t->d_pos);
    dfree(t->d_pidx);
    dfree(t->d_cd);
    dfree(t->d_cv);
    dfree(t->d_lo);
    dfree(t->d_hi);
    dfree(t->d_box);
    dfree(t->d_view);
    delete t;
}

// pinned host staging reused across builds (pinning is slow); builds on one device are serialised by its mutex
static constexpr int KD_MAX_DEV = 64;
static std::mutex g_build_mu[KD_MAX_DEV];
struct Pinned {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t bytes) {
        if (bytes > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) return nullptr;
            cap = bytes;
        }
        return p;
    }
};
static Pinned g_pin_nodes[KD_MAX_DEV], g_pin_ch[KD_MAX_DEV];

KdTree *kd_tree_build(const float *d_rows, int n, int dd, int bs, hipStream_t stream) {
    const auto t0 = std::chrono::steady_clock::now();
    int kdev = 0;
    if (hipGetDevice(&kdev) != hipSuccess || kdev < 0 || kdev >= KD_MAX_DEV) kdev = 0;
    std::lock_guard<std::mutex> build_lk(g_build_mu[kdev]);
    KdTree *t = new KdTree();
    t->n = n;
    t->dd = dd;
    t->bs = std::max(1, bs);
    struct Guard {  // returns the build's device scratch to the block cache on every exit path, once idle
        std::vector<void *> dev;
        hipStream_t s;
        ~Guard() {
            if (!dev.empty()) (void)hipStreamSynchronize(s);  // an error exit may leave work queued on it
            for (void *p : dev) dfree(p);
        }
    } g;
    g.s = stream;
    auto fail = [&]() -> KdTree * {
        kd_tree_destroy(t);
        return nullptr;
    };
#define KD_CHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) {                                                                \
            set_error(std::string("kd-tree build: ") + #expr + ": " + hipGetErrorString(_e)); \
            return fail();                                                                     \
        }                                                                                      \
    } while (0)
#define KD_PIN(ptr, pool, bytes)                                       \
    do {                                                               \
        ptr = (decltype(ptr))pool.get(bytes);                          \
        if (!ptr) {                                                    \
            set_error("kd-tree build: pinned host allocation failed"); \
            return fail();                                             \
        }                                                              \
    } while (0)
    const size_t nn1 = (size_t)std::max(n, 1);
    KD_CHECK(dmalloc((void **)&t->d_pos, nn1 * 4));
    KD_CHECK(dmalloc((void **)&t->d_pidx, nn1 * 4));
    KD_CHECK(dmalloc((void **)&t->d_cd, nn1 * 4));
    KD_CHECK(dmalloc((void **)&t->d_cv, nn1 * 4));
    KD_CHECK(dmalloc((void **)&t->d_lo, nn1 * 4));
    KD_CHECK(dmalloc((void **)&t->d_hi, nn1 * 4));
    KD_CHECK(dmalloc((void **)&t->d_box, (size_t)2 * std::max(dd, 1) * 4));
    KD_CHECK(dmalloc((void **)&t->d_view, sizeof(KdOrder)));
    KD_CHECK(hipMemsetAsync(t->d_cd, 0, nn1 * 4, stream));
    KD_CHECK(hipMemsetAsync(t->d_cv, 0, nn1 * 4, stream));
    KD_CHECK(hipMemsetAsync(t->d_lo, 0, nn1 * 4, stream));
    KD_CHECK(hipMemsetAsync(t->d_hi, 0, nn1 * 4, stream));
    KD_CHECK(hipMemsetAsync(t->d_box, 0, (size_t)2 * std::max(dd, 1) * 4, stream));
    hipLaunchKernelGGL(kd_pos_kernel, dim3((unsigned)((nn1 + 255) / 256)), dim3(256), 0, stream, n,
                       (const int *)nullptr, t->d_pidx);  // SkeletonTree: pidx[i] = i
    KD_CHECK(hipGetLastError());
    if (n > t->bs) {
        // The shape is implicit (node [s, e) splits at s + (e - s) / 2), so every level is planned here, before any
        // data exists: the levels of nodes > KD_SUB points (each node by kd_median_big_kernel), then the subtrees
        // of <= KD_SUB points (kd_subtree_waves_kernel).  Nothing comes back to the host until the tree is done.
        std::vector<std::vector<std::pair<int, int>>> levels;
        std::vector<std::pair<int, int>> level, next, deferred;
        (n <= KD_SUB ? deferred : level).emplace_back(0, n);
        while (!level.empty()) {
            levels.push_back(level);  // sorted by size, descending: the big ones (> KD_CH points) are a prefix
            next.clear();
            for (const auto &nd : level) {
                const int s = nd.first, e = nd.second, m = s + (e - s) / 2;
                if (m - s > t->bs) (m - s <= KD_SUB ? deferred : next).emplace_back(s, m);
                if (e - m > t->bs) (e - m <= KD_SUB ? deferred : next).emplace_back(m, e);
            }
            std::stable_sort(next.begin(), next.end(), [](const std::pair<int, int> &a, const std::pair<int, int> &b) {
                return a.second - a.first > b.second - b.first;
            });
            level.swap(next);
        }
        const int nlev = (int)levels.size();
        std::vector<int> node_off(nlev + 1, 0), ch_off(nlev + 1, 0), nbig(nlev, 0);
        for (int L = 0; L < nlev; L++) {
            int nch = 0;
            for (size_t i = 0; i < levels[L].size(); i++) {
                const int s = levels[L][i].first, e = levels[L][i].second;
                if (e - s > KD_CH) {
                    nbig[L] = (int)i + 1;
                    nch += (e - s + KD_CH - 1) / KD_CH;
                }
            }
            node_off[L + 1] = node_off[L] + (int)levels[L].size();
            ch_off[L + 1] = ch_off[L] + nch;
        }
        const int n_nodes = node_off[nlev] + (int)deferred.size(), n_ch = ch_off[nlev];
        KdNodeDev *h_nodes;
        KdChunk *h_ch;
        KD_PIN(h_nodes, g_pin_nodes[kdev], (size_t)std::max(n_nodes, 1) * sizeof(KdNodeDev));
        KD_PIN(h_ch, g_pin_ch[kdev], (size_t)std::max(n_ch, 1) * sizeof(KdChunk));
        int max_nn = 1, max_big = 1;
        for (int L = 0; L < nlev; L++) {
            int c = ch_off[L];
            for (size_t i = 0; i < levels[L].size(); i++) {
                const int s = levels[L][i].first, e = levels[L][i].second;
                h_nodes[node_off[L] + i] = KdNodeDev{s, e};
                if ((int)i < nbig[L])
                    for (int x = s; x < e; x += KD_CH) h_ch[c++] = KdChunk{(int)i, x, std::min(e, x + KD_CH)};
            }
            max_nn = std::max(max_nn, (int)levels[L].size());
            max_big = std::max(max_big, nbig[L]);
        }
        for (size_t i = 0; i < deferred.size(); i++)
            h_nodes[node_off[nlev] + i] = KdNodeDev{deferred[i].first, deferred[i].second};
        float *d_keys = nullptr;
        unsigned *d_omin = nullptr, *d_omax = nullptr;
        int *d_cut = nullptr, *d_lpos = nullptr, *d_rpos = nullptr;
        KdChunk *d_ch = nullptr;
        KdNodeDev *d_nodes = nullptr;
        KD_CHECK(dmalloc((void **)&d_nodes, (size_t)std::max(n_nodes, 1) * sizeof(KdNodeDev)));
        g.dev.push_back(d_nodes);
        KD_CHECK(hipMemcpyAsync(d_nodes, h_nodes, (size_t)n_nodes * sizeof(KdNodeDev), hipMemcpyHostToDevice, stream));
        if (nlev > 0) {
            KD_CHECK(dmalloc((void **)&d_keys, nn1 * 4));
            g.dev.push_back(d_keys);
            KD_CHECK(dmalloc((void **)&d_lpos, nn1 * 4));
            g.dev.push_back(d_lpos);
            KD_CHECK(dmalloc((void **)&d_rpos, nn1 * 4));
            g.dev.push_back(d_rpos);
            KD_CHECK(dmalloc((void **)&d_omin, (size_t)max_big * dd * 4));
            g.dev.push_back(d_omin);
            KD_CHECK(dmalloc((void **)&d_omax, (size_t)max_big * dd * 4));
            g.dev.push_back(d_omax);
            KD_CHECK(dmalloc((void **)&d_cut, (size_t)max_nn * 4));
            g.dev.push_back(d_cut);
            KD_CHECK(dmalloc((void **)&d_ch, (size_t)std::max(n_ch, 1) * sizeof(KdChunk)));
            g.dev.push_back(d_ch);
            if (n_ch > 0)
                KD_CHECK(hipMemcpyAsync(d_ch, h_ch, (size_t)n_ch * sizeof(KdChunk), hipMemcpyHostToDevice, stream));
        }
        for (int L = 0; L < nlev; L++) {
            const int nn = (int)levels[L].size(), nb = nbig[L], nch = ch_off[L + 1] - ch_off[L];
            const KdNodeDev *lv = d_nodes + node_off[L];
            const KdChunk *lch = d_ch + ch_off[L];
            float *box_out = L == 0 ? t->d_box : nullptr;
            if (nb > 0) {
                KD_CHECK(hipMemsetAsync(d_omin, 0xff, (size_t)nb * dd * 4, stream));
                KD_CHECK(hipMemsetAsync(d_omax, 0x00, (size_t)nb * dd * 4, stream));
                hipLaunchKernelGGL(kd_spread_big_kernel, dim3((nch + 3) / 4), dim3(256), 0, stream, d_rows, dd,
                                   (const int *)t->d_pidx, lch, nch, d_omin, d_omax);
                KD_CHECK(hipGetLastError());
                hipLaunchKernelGGL(kd_select_big_kernel, dim3((nb + 3) / 4), dim3(256), 0, stream, dd, nb,
                                   (const unsigned *)d_omin, (const unsigned *)d_omax, d_cut, box_out);
                KD_CHECK(hipGetLastError());
                hipLaunchKernelGGL(kd_gather_kernel, dim3((nch + 3) / 4), dim3(256), 0, stream, d_rows, dd,
                                   (const int *)t->d_pidx, lch, nch, (const int *)d_cut, d_keys);
                KD_CHECK(hipGetLastError());
                box_out = nullptr;
            }
            if (nn > nb) {
                hipLaunchKernelGGL(kd_small_kernel, dim3((nn - nb + 3) / 4), dim3(256), 0, stream, d_rows, dd,
                                   (const int *)t->d_pidx, lv + nb, nn - nb, d_cut + nb, d_keys, box_out);
                KD_CHECK(hipGetLastError());
            }
            hipLaunchKernelGGL(kd_median_big_kernel, dim3(nn), dim3(64 * KD_MW), 0, stream, d_keys, t->d_pidx, lv,
                               (const int *)d_cut, d_lpos, d_rpos, t->d_cd, t->d_cv);
            KD_CHECK(hipGetLastError());
            t->levels++;
        }
        if (!deferred.empty()) {
            const KdNodeDev *dn = d_nodes + node_off[nlev];
            if (nlev == 0) {  // the whole tree is one subtree: the enclosing box comes from a root spread
                int *d_cut1 = nullptr;
                float *d_keys1 = nullptr;
                KD_CHECK(dmalloc((void **)&d_cut1, 4));
                g.dev.push_back(d_cut1);
                KD_CHECK(dmalloc((void **)&d_keys1, nn1 * 4));
                g.dev.push_back(d_keys1);
                hipLaunchKernelGGL(kd_small_kernel, dim3(1), dim3(256), 0, stream, d_rows, dd, (const int *)t->d_pidx,
                                   dn, 1, d_cut1, d_keys1, t->d_box);
                KD_CHECK(hipGetLastError());
            }
            const int nd = (int)deferred.size();
            hipLaunchKernelGGL(kd_subtree_waves_kernel, dim3(nd), dim3(64 * KD_SW), 0, stream, d_rows, dd, t->d_pidx,
                               dn, t->bs, t->d_cd, t->d_cv);
            KD_CHECK(hipGetLastError());
            int maxd = 0;  // levels: the big ones + the deepest subtree's
            for (const auto &d : deferred) {
                int depth = 0;
                for (int c = d.second - d.first; c > t->bs; c = (c + 1) / 2) depth++;
                maxd = std::max(maxd, depth);
            }
            t->levels += maxd;
        }
        hipLaunchKernelGGL(kd_bounds_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, t->bs,
                           (const int *)t->d_cd, (const float *)t->d_cv, (const float *)t->d_box, dd, t->d_lo,
                           t->d_hi);
        KD_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(kd_pos_kernel, dim3((unsigned)((nn1 + 255) / 256)), dim3(256), 0, stream, n,
                       (const int *)t->d_pidx, t->d_pos);
    KD_CHECK(hipGetLastError());
    const KdOrder view = t->view();
    KD_CHECK(hipMemcpyAsync(t->d_view, &view, sizeof(KdOrder), hipMemcpyHostToDevice, stream));
    KD_CHECK(hipStreamSynchronize(stream));  // the scratch is freed on return; the caller gets a finished tree
#undef KD_CHECK
#undef KD_PIN
    t->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return t;
}

int kd_tree_positions(const KdTree *t, int32_t *pos) {
    if (!t || t->n == 0) return 0;
    TILER_HIP_CHECK(hipMemcpy(pos, t->d_pos, (size_t)t->n * 4, hipMemcpyDeviceToHost));
    return 0;
}

// ------------------------------------------------------------------------------------------
// pruning check + exact replay
// ------------------------------------------------------------------------------------------
// One thread per query: ANN visits result c iff every far-child box distance on its path is below the k-th key
// current at that check.  That key is >= D_k (the final k-th distance) throughout, and > D_k while c is a tie at
// D_k not yet inserted, so box < D_k (or <= D_k for such a tie) vouches for c; otherwise -> replay.
__global__ __launch_bounds__(256) void kd_verify_kernel(KdOrder o, KdFixArgs a) {
    const long q = (long)blockIdx.x * 256 + threadIdx.x;
    if (q >= a.nq) return;
    if (a.done && a.done[q]) return;
    const float *qr = a.q + q * o.dd;
    const float Dk = a.err[q * a.k + a.k - 1];
    const int i0 = a.idx[q * a.k];
    if (i0 < 0 || !(Dk < FLT_MAX)) return;  // empty dataset or fewer than k points: nothing to vouch for
    const float rb = a.rootbox[q];
    bool ok = true;
    for (int j = 0; j < a.k && ok; j++) {
        const int c = a.idx[q * a.k + j];
        if ((unsigned)c >= (unsigned)o.n) {
            ok = false;
            break;
        }
        const float fb = kd_path_far_box(o, qr, o.pos[c], rb);
        const float dc = a.err[q * a.k + j];
        ok = fb < Dk || (fb <= Dk && dc == Dk);
    }
    if (!ok || a.force_replay) a.list[atomicAdd(a.count, 1)] = (int)q;
}

// annkSearch replayed exactly: kd_replay_query (kdorder_dev.hpp), one thread per listed query
template <int K>
__global__ __launch_bounds__(64) void kd_replay_kernel(KdOrder o, KdFixArgs a) {
    const int count = *a.count;
    for (int li = blockIdx.x * 64 + threadIdx.x; li < count; li += gridDim.x * 64) {
        const long q = a.list[li];
        const int best = kd_replay_query<K>(o, a.rows, a.q + q * o.dd, a.k, a.idx + q * a.k, a.err + q * a.k);
        if (a.m_tile) {
            a.m_tile[q] = best >= 0 ? a.tr_tile[best] : -1;
            a.m_pal[q] = best >= 0 ? a.tr_pal[best] : -1;
            const int at = best >= 0 ? a.tr_attr[best] : 0;
            a.m_hm[q] = (at & 1) != 0;
            a.m_vm[q] = (at & 2) != 0;
        }
    }
}

// annkPriSearch replayed exactly (ANN.dll 0x1800121a0-0x18001257f, ANNkd_split::ann_pri_search 0x180012580,
// ANNkd_leaf::ann_pri_search 0x180012670, ANNpr_queue::insert 0x180008fc0; extr_min inlined at 0x1800122d0): the
// root enters a binary min-heap with its box distance; each extracted node whose key * (1 + eps)^2 is below the
// current best descends to a leaf on q's side, pushing every far child with key (cut_diff^2 - box_diff^2) + box
// (box_diff = maxss(bound difference, 0)); the leaf scan and the k = 1 ANNmin_k insertion are annkSearch's.  One
// thread per query; the heap lives in global scratch (n + 1 entries per query, ANN's pr_queue(n_pts) size).
struct PriEntry {
    float key;
    int s, e;  // the node: leaf positions [s, e)
};

__global__ __launch_bounds__(64) void kd_pri_kernel(KdOrder o, const float *__restrict__ rows,
                                                    const float *__restrict__ q, int nq, float eps,
                                                    PriEntry *__restrict__ heap, int *__restrict__ out_idx,
                                                    float *__restrict__ out_err, const uint8_t *__restrict__ only,
                                                    const int *__restrict__ tcnt, const int *__restrict__ tlist) {
    const int qi = blockIdx.x * 64 + threadIdx.x;
    if (qi >= nq) return;
    if (only && !only[qi]) return;  // resolved by kd_pri_resolve_kernel
    const bool sim = only && only[qi] == 2;  // heap order only: the first extracted leaf holding a target wins
    PriEntry *pq = heap + (size_t)qi * ((size_t)o.n + 1);  // pq[1..n]
    const float *qr = q + (long)qi * o.dd;
    float max_err = eps + 1.0f;
    max_err = max_err * max_err;
    int hn = 0;
    auto insert = [&](float kv, int s, int e) {  // ANNpr_queue::insert: sift up while the parent's key > kv
        int r = ++hn;
        while (r > 1) {
            const int p = r >> 1;
            if (pq[p].key <= kv) break;
            pq[r] = pq[p];
            r = p;
        }
        pq[r] = PriEntry{kv, s, e};
    };
    int cnt = 0, best_i = -1;
    float best = FLT_MAX;
    insert(kd_root_box(o, qr), 0, o.n);
    int nt = 0;
    const int *tl = nullptr;
    if (sim) {
        nt = tcnt[qi];
        tl = tlist + (long)qi * 64;  // KD_PRI_CAP
    }
    while (hn > 0) {
        const PriEntry top = pq[1];  // extr_min
        const float kn = pq[hn].key;
        hn--;
        int p = 1, r = 2;
        while (r <= hn) {
            if (r < hn && pq[r].key > pq[r + 1].key) r++;
            if (kn <= pq[r].key) break;
            pq[p] = pq[r];
            p = r;
            r = p << 1;
        }
        pq[p] = pq[hn + 1];
        if (!sim && top.key * max_err >= (cnt ? best : FLT_MAX)) break;
        const float box = top.key;
        int s = top.s, e = top.e;
        while (e - s > o.bs) {  // ANNkd_split::ann_pri_search: push the far child, continue on q's side (same box)
            const int m = s + ((e - s) >> 1);
            const float qd = qr[o.cd[m]];
            const float cut_diff = qd - o.cv[m];
            if (cut_diff < 0.0f) {
                float box_diff = o.lo[m] - qd;
                box_diff = box_diff > 0.0f ? box_diff : 0.0f;  // maxss(box_diff, 0)
                insert((cut_diff * cut_diff - box_diff * box_diff) + box, m, e);
                e = m;
            } else {
                float box_diff = qd - o.hi[m];
                box_diff = box_diff > 0.0f ? box_diff : 0.0f;
                insert((cut_diff * cut_diff - box_diff * box_diff) + box, s, m);
                s = m;
            }
        }
        if (sim) {  // the leaf [s, e): its lowest-position target, if any, is the answer
            int win = -1, wp = 0x7fffffff;
            for (int j = 0; j < nt; j++) {
                const int t = tl[j], pt = o.pos[t];
                if (pt >= s && pt < e && pt < wp) {
                    wp = pt;
                    win = t;
                }
            }
            if (win >= 0) {
                out_idx[qi] = win;  // out_err: the minimum, written by kd_pri_resolve_kernel
                return;
            }
            continue;
        }
        float min_dist = cnt ? best : FLT_MAX;  // ANNkd_leaf::ann_pri_search
        for (int lp = s; lp < e; lp++) {
            const int pt = o.pidx[lp];
            const float *pp = rows + (long)pt * o.dd;
            float dist;
            if (kd_leaf_dist(qr, pp, o.dd, min_dist, dist)) {  // ANNmin_k::insert with k = 1: an equal key lands in slot 1 and is dropped
                if (!cnt || best > dist) {
                    best = dist;
                    best_i = pt;
                }
                cnt = 1;
                min_dist = best;
            }
        }
    }
    out_idx[qi] = cnt ? best_i : -1;
    out_err[qi] = cnt ? best : FLT_MAX;
}

// The priority search's answer without the replay (eps = 0, k = 1).  Leaves leave the heap in ascending order of
// their entry key -- the box value after the last far step on the leaf's root path, i.e. kd_path_far_box's maximum
// (the root box without a far step): a node's entry is pushed by a chain whose key is <= its own, so it is in the
// heap before any larger key is extracted.  Let D be the exact minimum distance and S the points at D.  A point of S
// whose entry key is < D is visited (termination needs an extracted key >= the best so far >= D) and inserted; every
// point of S with a larger entry key comes later and cannot replace it (ANNmin_k keeps the first of equal keys).  So
// the answer is the point of S with the smallest entry key below D, the bucket order deciding inside one leaf.  A
// query falls back to the replay when that is not decided this way: no point of S below D, two leaves with the same
// smallest key (the heap's own tie order), or more than KD_PRI_CAP points within the annkSearch distance.
static constexpr int KD_PRI_CAP = 64;

// every point within d0[q] (annkSearch's distance, >= D) of query q -> list[q][.] with its exact distance
__global__ __launch_bounds__(256) void kd_pri_ties_kernel(const float *__restrict__ rows, int n, int dd,
                                                         const float *__restrict__ q, int nq,
                                                         const float *__restrict__ d0, int *__restrict__ cnt,
                                                         int *__restrict__ list, float *__restrict__ ldist) {
    for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < n; r += (long)gridDim.x * 256)
        for (int qi = blockIdx.y; qi < nq; qi += gridDim.y) {
            const float lim = d0[qi];
            const float *qr = q + (long)qi * dd;
            const float *pr = rows + r * dd;
            float dist = 0.0f;
            int d;
            for (d = 0; d < dd; d++) {
                const float t = qr[d] - pr[d];
                dist = dist + t * t;
                if (dist > lim) break;  // partial sums only grow
            }
            if (d < dd) continue;
            const int slot = atomicAdd(cnt + qi, 1);
            if (slot < KD_PRI_CAP) {
                list[(long)qi * KD_PRI_CAP + slot] = (int)r;
                ldist[(long)qi * KD_PRI_CAP + slot] = dist;
            }
        }
}

// one wave per query: the rule above, or the query flagged for kd_pri_kernel
__global__ __launch_bounds__(64) void kd_pri_resolve_kernel(KdOrder o, const float *__restrict__ q, int nq,
                                                            int *__restrict__ cnt, int *__restrict__ list,
                                                            const float *__restrict__ ldist, int *__restrict__ out_idx,
                                                            float *__restrict__ out_err, uint8_t *__restrict__ flag) {
    const int qi = blockIdx.x, lane = threadIdx.x;
    const float *qr = q + (long)qi * o.dd;
    const int c = cnt[qi];
    if (c <= 0 || c > KD_PRI_CAP) {  // uniform
        if (lane == 0) flag[qi] = 1;
        return;
    }
    const int my_i = lane < c ? list[(long)qi * KD_PRI_CAP + lane] : -1;
    const float my_d = lane < c ? ldist[(long)qi * KD_PRI_CAP + lane] : INFINITY;
    float dm = my_d;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dm = fminf(dm, __shfl_xor(dm, off, 64));
    const bool in_s = lane < c && my_d == dm;
    const float rb = kd_root_box_wave(o, qr, lane);
    // entry keys of S's members, two per pass (one half-wave each)
    float my_ek = INFINITY;
    unsigned long long m = __ballot(in_s);
    while (m) {  // uniform
        const int a0 = __builtin_ctzll(m);
        m &= m - 1;
        int a1 = -1;
        if (m) {
            a1 = __builtin_ctzll(m);
            m &= m - 1;
        }
        const int mine = (lane >> 5) ? a1 : a0;
        const int ci = __shfl(my_i, mine < 0 ? 0 : mine, 64);
        const float w = kd_half_path_far_box(o, qr, mine < 0 ? 0 : o.pos[ci], rb, lane);
        const float ek = w == -INFINITY ? rb : w;
        const float e0 = __shfl(ek, 0, 64), e1 = __shfl(ek, 32, 64);
        if (lane == a0) my_ek = e0;
        if (a1 >= 0 && lane == a1) my_ek = e1;
    }
    // the smallest entry key, then its members' leaves (start positions, from the positions alone)
    float ekm = my_ek;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ekm = fminf(ekm, __shfl_xor(ekm, off, 64));
    const bool cand = in_s && my_ek == ekm;
    int leaf = 0x7fffffff, p = 0x7fffffff;
    if (cand) {
        p = o.pos[my_i];
        int s = 0, e = o.n;
        while (e - s > o.bs) {
            const int mm = s + ((e - s) >> 1);
            if (p < mm)
                e = mm;
            else
                s = mm;
        }
        leaf = s;
    }
    int lmin = leaf, lmax = cand ? leaf : -1, pmin = p;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lmin = min(lmin, __shfl_xor(lmin, off, 64));
        lmax = max(lmax, __shfl_xor(lmax, off, 64));
        pmin = min(pmin, __shfl_xor(pmin, off, 64));
    }
    const bool decided = ekm < dm && lmin == lmax;  // uniform
    // smallest key below D but held by several leaves: the heap's order among them decides -- kd_pri_kernel simulates
    // the heap alone (flag 2: no leaf scans; every entry below D is extracted before the search could stop) up to the
    // first of these leaves; the candidates go to the front of the query's list, their count to cnt[qi]
    const bool heap_tie = ekm < dm && lmin != lmax;
    if (lane == 0) flag[qi] = decided ? 0 : heap_tie ? 2 : 1;
    if (decided && cand && p == pmin) {
        out_idx[qi] = my_i;
        out_err[qi] = dm;
    }
    if (heap_tie) {  // uniform; every lane read its list entry above
        const unsigned long long cm = __ballot(cand);
        if (cand) {
            const int rank = __popcll(cm & ((1ull << lane) - 1));
            list[(long)qi * KD_PRI_CAP + rank] = my_i;
        }
        if (lane == 0) {
            cnt[qi] = __popcll(cm);
            out_err[qi] = dm;
        }
    }
}

int kd_pri_resolve(const KdTree *t, const float *d_rows, const float *d_q, int nq, const float *d_err0, void *aux,
                   int *d_idx, float *d_err, uint8_t *flag, hipStream_t stream) {
    if (!t || nq <= 0) return 0;
    int *cnt = (int *)aux;
    int *list = cnt + nq;
    float *ldist = (float *)(list + (size_t)nq * KD_PRI_CAP);
    KTimer tm("kd_pri_resolve", stream);
    TILER_HIP_CHECK(hipMemsetAsync(cnt, 0, (size_t)nq * sizeof(int), stream));
    const dim3 grid((unsigned)std::min<long>(((long)t->n + 255) / 256, 2048), (unsigned)std::min(nq, 64));
    hipLaunchKernelGGL(kd_pri_ties_kernel, grid, dim3(256), 0, stream, d_rows, t->n, t->dd, d_q, nq, d_err0, cnt, list,
                       ldist);
    hipLaunchKernelGGL(kd_pri_resolve_kernel, dim3((unsigned)nq), dim3(64), 0, stream, t->view(), d_q, nq,
                       cnt, list, (const float *)ldist, d_idx, d_err, flag);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

size_t kd_pri_aux_bytes(int nq) { return (size_t)std::max(nq, 0) * (1 + 2 * KD_PRI_CAP) * 4; }

size_t kd_pri_heap_bytes(const KdTree *t, int nq) {
    return t ? (size_t)std::max(nq, 0) * ((size_t)t->n + 1) * sizeof(PriEntry) : 0;
}

int kd_pri_search(const KdTree *t, const float *d_rows, const float *d_q, int nq, float eps, void *heap, int *d_idx,
                  float *d_err, hipStream_t stream, const uint8_t *only, const void *aux) {
    if (!t || nq <= 0) return 0;
    if (!heap) {
        set_error("kd_pri_search: no heap scratch");
        return -1;
    }
    KTimer tm("kd_pri", stream);
    hipLaunchKernelGGL(kd_pri_kernel, dim3((unsigned)((nq + 63) / 64)), dim3(64), 0, stream, t->view(), d_rows, d_q,
                       nq, eps, (PriEntry *)heap, d_idx, d_err, only, aux ? (const int *)aux : nullptr,
                       aux ? (const int *)aux + nq : nullptr);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

// one wave per query: coalesced row read, the outside-the-box terms in parallel, then their sequential fp32 sum
// in dimension order (a term inside the box is +0 and leaves the running sum unchanged, so only the others are
// added, by one lane, in order)
// done / count (or null): the search's per-query verify flags and replay count, cleared here (saves two memsets)
__global__ __launch_bounds__(256) void kd_rootbox_kernel(KdOrder o, const float *__restrict__ q, int nq,
                                                         float *__restrict__ out, uint8_t *__restrict__ done,
                                                         int *__restrict__ count) {
    const int lane = threadIdx.x & 63;
    if (count && blockIdx.x == 0 && threadIdx.x == 0) *count = 0;
    if (done)
        for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nq; i += (long)gridDim.x * 256) done[i] = 0;
    for (long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6); i < nq; i += (long)gridDim.x * 4) {
        float rb = 0.0f;
        for (int d0 = 0; d0 < o.dd; d0 += 64) {
            const int d = d0 + lane;
            float t = 0.0f;
            bool outside = false;
            if (d < o.dd) {
                const float v = q[i * o.dd + d], lo = o.box_lo[d], hi = o.box_hi[d];
                if (v < lo) {
                    t = lo - v;
                    outside = true;
                } else if (v > hi) {
                    t = v - hi;
                    outside = true;
                }
                t = t * t;
            }
            unsigned long long m = __ballot(outside);
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1;
                rb = rb + __shfl(t, src, 64);
            }
        }
        if (lane == 0) out[i] = rb;
    }
}

int kd_root_boxes(const KdTree *t, const float *d_q, int nq, float *rootbox, hipStream_t stream, uint8_t *done,
                  int *count) {
    if (!t || nq <= 0) return 0;
    KTimer tm("kd_verify", stream);
    hipLaunchKernelGGL(kd_rootbox_kernel, dim3((unsigned)std::min<long>(8192, (nq + 3) / 4)), dim3(256), 0, stream,
                       t->view(), d_q, nq, rootbox, done, count);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

// the replay alone, for queries some earlier kernel already checked and listed in a.list / *a.count
int kd_replay_listed(const KdTree *t, const KdFixArgs &a, hipStream_t stream) {
    if (!t || a.nq <= 0) return 0;
    if (a.k > 32) {
        set_error("kd replay: k > 32");
        return -1;
    }
    const KdOrder o = t->view();
    KTimer tm("kd_replay", stream);
    const dim3 grid(std::min(64, (a.nq + 63) / 64));  // grid-stride over the device-side count
    if (a.k <= 1)
        hipLaunchKernelGGL(kd_replay_kernel<1>, grid, dim3(64), 0, stream, o, a);
    else if (a.k <= 8)
        hipLaunchKernelGGL(kd_replay_kernel<8>, grid, dim3(64), 0, stream, o, a);
    else
        hipLaunchKernelGGL(kd_replay_kernel<32>, grid, dim3(64), 0, stream, o, a);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

int kd_verify_and_replay(const KdTree *t, const KdFixArgs &a, hipStream_t stream) {
    if (!t || t->n <= t->bs || a.nq <= 0) return 0;  // a single bucket: no pruning, position order is exact
    if (a.k > 32) {
        set_error("kd replay: k > 32");
        return -1;
    }
    const KdOrder o = t->view();
    {
        KTimer tm("kd_verify", stream);
        hipLaunchKernelGGL(kd_verify_kernel, dim3((a.nq + 255) / 256), dim3(256), 0, stream, o, a);
    }
    TILER_HIP_CHECK(hipGetLastError());
    {
        KTimer tm("kd_replay", stream);
        const dim3 grid(64);  // grid-stride over the device-side count: no host round trip
        if (a.k <= 1)
            hipLaunchKernelGGL(kd_replay_kernel<1>, grid, dim3(64), 0, stream, o, a);
        else if (a.k <= 8)
            hipLaunchKernelGGL(kd_replay_kernel<8>, grid, dim3(64), 0, stream, o, a);
        else
            hipLaunchKernelGGL(kd_replay_kernel<32>, grid, dim3(64), 0, stream, o, a);
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tiler

// nn_search.hip -- exact nearest-neighbour search over fp32 descriptors on gfx950 (MI355X).
//
// Replaces ANN.dll's kd-tree search (called at main.pas:3830 and 4027).  The
// result must equal an exhaustive scan of the reference distance
//     dist(q, c) = fp32 sum over d of (q_d - c_d)^2, dimension order, every op rounded, no FMA
// with equal distances resolved to the lowest dataset index.  That sum is not a GEMM, so the
// search runs in three kernels:
//   1. nn_shortlist_kernel: keys = ||c||^2 - 2 q.c on the matrix cores (v_mfma_f32_32x32x16_f16 on
//      fp16-rounded operands, fp32 accumulate).  Every lane keeps the L smallest keys of its
//      query column; nothing Q x M ever reaches HBM.
//   2. nn_rescore_kernel: per query, a rigorous bound E on |key - exact key| (norms of the fp16
//      residuals + accumulation and rounding terms, DESIGN.md "Exactness argument") gives a
//      threshold T >= the key of the exact winner; every kept candidate with key <= T is rescored
//      with the reference fp32 sequential distance and the winner picked by (dist, index).
//      If a lane's list was full below T (a candidate might have been dropped) the query is queued.
//   3. nn_exact_kernel: exhaustive reference-order scan for queued queries (and k > 8).
// Small-integer datasets (the 64-d palette-index preselection, main.pas:3779/3830) make the MFMA
// keys exact; the same kernels then return exact (key, index) order with no margin.
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>

#include "nn_search.hpp"
#include "kdorder_dev.hpp"
#include "nn_dev.hpp"
#include "orbit.hpp"
#include "orbit_map_gen.hpp"
#include "psyv.hpp"

#pragma clang fp contract(off)

namespace tiler {

enum { QF_INT = 1, QF_BAD = 2 };

// ------------------------------------------------------------------------------------------
// prep: fp32 rows -> fp16 MFMA fragments [blk][s][lane][8] + norms + bounds
//   lane l of block b holds row b*32 + (l & 31), k = s*16 + 8*(l >> 5) + j   (A and B maps coincide)
// ------------------------------------------------------------------------------------------
struct PrepArgs {
    const float *rows;
    long n;
    int d, S;
    float scale;
    half8 *frag;
    float *nc;      // dataset only: accumulator-row order
    float *seed;    // dataset only: -||c||^2/2 in accumulator-row order (shortlist accumulator seed)
    QStat *qstat;   // queries only
    DsStat *ds;     // dataset only
    int perm;       // dataset only: A-operand row i holds candidate blk*32 + row_perm(i)
};

// Candidate -> A-operand row permutation (swap bits 0 and 2 of the row).  The 4 mirror candidates of
// one tile are consecutive indices; unpermuted they all land in the same accumulator lane (rows
// 4h..4h+3), so a 4-way near-tie fills that lane's list.  Swapping bits 0 and 2 spreads them 2+2 over
// the two half-waves.  Involution; identity for exact-integer datasets (arrival order = index order).
__device__ __forceinline__ int row_perm(int i) { return (i & ~5) | ((i & 1) << 2) | ((i >> 2) & 1); }


__global__ __launch_bounds__(256) void prep_rows_kernel(PrepArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
    const long nblk = (a.n + 31) / 32;
    double t_n2 = 0.0, t_h2 = 0.0, t_e2 = 0.0, t_ab = 0.0;
    int t_ni = 0, t_bd = 0;
    for (long blk = (long)blockIdx.x * 4 + wave; blk < nblk; blk += (long)gridDim.x * 4) {
        const long r = blk * 32 + (a.perm ? row_perm(lane & 31) : (lane & 31));
        const bool valid = r < a.n;
        double s2 = 0, sh = 0, se = 0, mabs = 0;
        int notint = 0, bad = 0;
        // the lane's 8 consecutive values of each k-step: two 16-byte loads when the rows allow it (d % 8 == 0, 32-byte
        // aligned base), each value alone otherwise; the values and everything computed from them are the same
        const bool vec = (a.d & 7) == 0 && (((uintptr_t)a.rows) & 31) == 0;
        for (int s = 0; s < a.S; s++) {
            half8 hv;
            float vv[8];
            const int k0 = s * 16 + 8 * h;
            if (vec) {
                float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
                if (valid && k0 < a.d) {
                    const float4 *src = reinterpret_cast<const float4 *>(a.rows + r * a.d + k0);
                    x0 = src[0];
                    x1 = src[1];
                }
                vv[0] = x0.x; vv[1] = x0.y; vv[2] = x0.z; vv[3] = x0.w;
                vv[4] = x1.x; vv[5] = x1.y; vv[6] = x1.z; vv[7] = x1.w;
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++) vv[j] = (valid && k0 + j < a.d) ? a.rows[r * a.d + k0 + j] : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float v = vv[j];
                const float vs = v * a.scale;
                _Float16 vh = (_Float16)vs;
                if (fabsf((float)vh) < 6.103515625e-05f) vh = (_Float16)0.0f;  // no fp16 subnormal operands
                hv[j] = vh;
                const double dv = vs, dh = (double)(float)vh;
                s2 += dv * dv;
                sh += dh * dh;
                se += (dv - dh) * (dv - dh);
                mabs = fmax(mabs, fabs((double)v));
                if (!(v == rintf(v)) || fabsf(v) > 2048.0f) notint = 1;
                if (!isfinite(vs) || fabsf(vs) > 65000.0f) bad = 1;
            }
            a.frag[(blk * a.S + s) * 64 + lane] = hv;
        }
        s2 += __shfl_xor(s2, 32, 64);
        sh += __shfl_xor(sh, 32, 64);
        se += __shfl_xor(se, 32, 64);
        mabs = fmax(mabs, __shfl_xor(mabs, 32, 64));
        notint |= __shfl_xor(notint, 32, 64);
        bad |= __shfl_xor(bad, 32, 64);
        if (a.qstat && h == 0 && valid) {
            QStat q;
            q.n2 = s2;
            q.hn = sqrt(sh);
            q.en = sqrt(se);
            q.flags = (notint ? 0 : QF_INT) | (bad ? QF_BAD : 0);
            q.pad = (int)fmin(mabs, 2e9);
            a.qstat[r] = q;
        }
        if (a.nc && h == 0) {
            const int rr = lane & 31;
            const int pos = ((rr >> 2) & 1) * 16 + ((rr & 3) | ((rr >> 3) << 2));
            a.nc[blk * 32 + pos] = valid ? (float)s2 : INFINITY;
            if (a.seed) a.seed[blk * 32 + pos] = valid ? -0.5f * (float)s2 : -INFINITY;
        }
        if (a.ds) {  // this thread's running maxima (all >= 0: the max of the bit patterns is the max of the values)
            if (valid) {
                t_n2 = fmax(t_n2, s2);
                t_h2 = fmax(t_h2, sh);
                t_e2 = fmax(t_e2, se);
                t_ab = fmax(t_ab, mabs);
                t_ni |= notint;
                t_bd |= bad;
            }
        }
    }
    if (a.ds) {  // one set of dataset atomics per workgroup (per wave and block they serialised on six addresses)
        __shared__ double r_d[4][4];
        __shared__ int r_i[4][2];
        const double m2 = wave_max_d(t_n2), mh = wave_max_d(t_h2), me = wave_max_d(t_e2), ma = wave_max_d(t_ab);
        const int ni = __any(t_ni), bd = __any(t_bd);
        if (lane == 0) {
            r_d[wave][0] = m2;
            r_d[wave][1] = mh;
            r_d[wave][2] = me;
            r_d[wave][3] = ma;
            r_i[wave][0] = ni;
            r_i[wave][1] = bd;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double v[4] = {0.0, 0.0, 0.0, 0.0};
            int f0 = 0, f1 = 0;
            for (int w = 0; w < 4; w++) {
                for (int x = 0; x < 4; x++) v[x] = fmax(v[x], r_d[w][x]);
                f0 |= r_i[w][0];
                f1 |= r_i[w][1];
            }
            atomicMax(&a.ds->max_n2_bits, (unsigned long long)__double_as_longlong(v[0]));
            atomicMax(&a.ds->max_h2_bits, (unsigned long long)__double_as_longlong(v[1]));
            atomicMax(&a.ds->max_e2_bits, (unsigned long long)__double_as_longlong(v[2]));
            atomicMax(&a.ds->max_abs_bits, (unsigned long long)__double_as_longlong(v[3]));
            if (f0) atomicOr(&a.ds->not_int, 1u);
            if (f1) atomicOr(&a.ds->bad, 1u);
        }
    }
}

// out[0] = max |v| (float bits), out[1] |= 1 if any value is not an integer
__global__ __launch_bounds__(256) void maxabs_kernel(const float *rows, long total, unsigned int *out) {
    float m = 0.0f;
    int ni = 0;
    auto fold = [&](float x) __attribute__((always_inline)) {
        const float v = fabsf(x);
        m = isfinite(v) ? fmaxf(m, v) : m;
        ni |= !(x == rintf(x));
    };
    const long stride = (long)gridDim.x * 256, g = (long)blockIdx.x * 256 + threadIdx.x;
    long i0 = 0;
    if ((((uintptr_t)rows) & 15) == 0) {  // 16-byte loads, two in flight per thread; the tail below
        const float4 *r4 = reinterpret_cast<const float4 *>(rows);
        const long n4 = total >> 2;
        long i = g;
        for (; i + stride < n4; i += 2 * stride) {
            const float4 x = r4[i], y = r4[i + stride];
            fold(x.x); fold(x.y); fold(x.z); fold(x.w);
            fold(y.x); fold(y.y); fold(y.z); fold(y.w);
        }
        if (i < n4) {
            const float4 x = r4[i];
            fold(x.x); fold(x.y); fold(x.z); fold(x.w);
        }
        i0 = n4 << 2;
    }
    for (long i = i0 + g; i < total; i += stride) fold(rows[i]);
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const bool any_ni = __any(ni);
    __shared__ float r_m[4];
    __shared__ int r_n[4];
    if ((threadIdx.x & 63) == 0) {
        r_m[threadIdx.x >> 6] = m;
        r_n[threadIdx.x >> 6] = any_ni;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // one pair of atomics per workgroup (one per wave serialised on the two words)
        const float mm = fmaxf(fmaxf(r_m[0], r_m[1]), fmaxf(r_m[2], r_m[3]));
        atomicMax(out, __float_as_uint(mm));
        if (r_n[0] | r_n[1] | r_n[2] | r_n[3]) atomicOr(out + 1, 1u);
    }
}

// ------------------------------------------------------------------------------------------
// 1. MFMA shortlist.  Workgroup = 4 waves; wave = 2 query blocks of 32 (64 queries); the
// candidate blocks of this split stream through a double-buffered LDS ring (CB blocks/stage).
// ------------------------------------------------------------------------------------------
// acc was seeded with -||c||^2/2, so acc = q.c - ||c||^2/2 and key = ||c||^2 - 2 q.c = -2 acc (exact
// scaling): the epilogue is a max tree plus one compare per 16 values, no per-value FMA.
template <int L>
__device__ __forceinline__ void scan_keys(const floatx16 &acc, int base, int h, int perm, float (&lk)[L],
                                          int (&li)[L]) {
    float mx = acc[0];
#pragma unroll
    for (int r = 1; r < 16; r++) mx = fmaxf(mx, acc[r]);
    const float thr = -0.5f * lk[L - 1];  // acc > thr  <=>  key < lk[L-1]
    if (mx > thr) {
#pragma unroll
        for (int r = 0; r < 16; r++)
            if (acc[r] > -0.5f * lk[L - 1]) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                list_insert<L>(lk, li, -2.0f * acc[r], base + (perm ? row_perm(row) : row));
            }
    }
}

// QB query blocks of 32 per wave (2: each A-fragment read feeds two MFMAs; 1: twice the waves for the same queries,
// for launches too small to give every SIMD more than one wave otherwise -- UseOne's k = 8 preselection)
template <int S, int L, int CB, int NW, int QB = 2>
__global__ __launch_bounds__(NW * 64, 2) void nn_shortlist_kernel(const half8 *__restrict__ cfrag,
                                                              const float *__restrict__ cnc, int nblk,
                                                              const half8 *__restrict__ qfrag, int nq,
                                                              int blk_per_split, int nsplit, int perm,
                                                              float *__restrict__ out_key, int *__restrict__ out_idx) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int FRAG_BYTES = CB * S * 1024;
    constexpr int BUF_BYTES = FRAG_BYTES + CB * 128;
    constexpr int NT = NW * 64;
    constexpr int PER_T = CB * S * 64 / NT;
    static_assert((CB * S * 64) % NT == 0, "stage must split evenly over the workgroup");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int nqblk = (nq + 31) / 32;
    const int qb0 = (blockIdx.x * NW + w) * QB;
    const int split = blockIdx.y;
    const int b_begin = split * blk_per_split;
    const int b_end = min(nblk, b_begin + blk_per_split);

    half8 bq[QB][S];
    // query blocks past the end compute on a clamped duplicate and are never written out
#pragma unroll
    for (int x = 0; x < QB; x++) {
        const long qa = min(qb0 + x, nqblk - 1);
#pragma unroll
        for (int s = 0; s < S; s++) bq[x][s] = qfrag[(qa * S + s) * 64 + lane];
    }
    float lk[QB][L];
    int li[QB][L];
#pragma unroll
    for (int x = 0; x < QB; x++)
#pragma unroll
        for (int i = 0; i < L; i++) {
            lk[x][i] = INFINITY;
            li[x][i] = -1;
        }

    const int nstage = (b_end > b_begin) ? (b_end - b_begin + CB - 1) / CB : 0;
    // LDS-DMA staging (global_load_lds_dwordx4): the fragment image is lane-linear, so each wave
    // copies 1 KiB pieces straight into LDS; the barrier at the end of a stage drains them.
    // Sources are clamped: blocks past b_end land in LDS but are never computed on.
    auto issue = [&](int st, int buf) {
        const int blk0 = b_begin + st * CB;
        const int nb = min(CB, b_end - blk0);
        const int last = nb * S * 64 - 1;
        const uint4 *src = reinterpret_cast<const uint4 *>(cfrag) + (long)blk0 * S * 64;
        char *dst = smem + buf * BUF_BYTES;
#pragma unroll
        for (int j = 0; j < PER_T; j++) glds16(src + min(j * NT + w * 64 + lane, last), dst + (j * NT + w * 64) * 16);
        if (w == 0 && lane < CB * 8)
            glds16(reinterpret_cast<const uint4 *>(cnc) + (long)blk0 * 8 + min(lane, nb * 8 - 1), dst + FRAG_BYTES);
    };

    if (nstage > 0) issue(0, 0);
    __syncthreads();
    for (int st = 0; st < nstage; st++) {
        const char *B = smem + (st & 1) * BUF_BYTES;
        // the stage's norms go to registers BEFORE the next DMA is issued: hipcc otherwise waits
        // vmcnt(0) (the DMA) at the first norm read, serialising the prefetch behind the compute
        float4 ncr[CB][4];
#pragma unroll
        for (int cb = 0; cb < CB; cb++)
#pragma unroll
            for (int i = 0; i < 4; i++) ncr[cb][i] = reinterpret_cast<const float4 *>(B + FRAG_BYTES)[cb * 8 + h * 4 + i];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (st + 1 < nstage) issue(st + 1, (st + 1) & 1);
#pragma unroll
        for (int cb = 0; cb < CB; cb++) {
            const int blk = b_begin + st * CB + cb;
            if (blk < b_end) {
                const float4 n0 = ncr[cb][0], n1 = ncr[cb][1], n2 = ncr[cb][2], n3 = ncr[cb][3];
                const floatx16 seed = {-0.5f * n0.x, -0.5f * n0.y, -0.5f * n0.z, -0.5f * n0.w,
                                       -0.5f * n1.x, -0.5f * n1.y, -0.5f * n1.z, -0.5f * n1.w,
                                       -0.5f * n2.x, -0.5f * n2.y, -0.5f * n2.z, -0.5f * n2.w,
                                       -0.5f * n3.x, -0.5f * n3.y, -0.5f * n3.z, -0.5f * n3.w};
                floatx16 acc[QB];
#pragma unroll
                for (int x = 0; x < QB; x++) acc[x] = seed;
#pragma unroll
                for (int s = 0; s < S; s++) {
                    const half8 av = reinterpret_cast<const half8 *>(B)[(cb * S + s) * 64 + lane];
#pragma unroll
                    for (int x = 0; x < QB; x++) acc[x] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[x][s], acc[x], 0, 0, 0);
                }
                const int base = blk * 32;
#pragma unroll
                for (int x = 0; x < QB; x++) scan_keys<L>(acc[x], base, h, perm, lk[x], li[x]);
            }
        }
        __syncthreads();  // vmcnt(0) + s_barrier: next stage's DMA landed, this stage's reads done
    }
    // partial lists: [q][split][h][L]
#pragma unroll
    for (int x = 0; x < QB; x++) {
        const int q = (qb0 + x) * 32 + (lane & 31);
        if (q < nq) {
            const long o = (((long)q * nsplit + split) * 2 + h) * L;
#pragma unroll
            for (int i = 0; i < L; i++) {
                out_key[o + i] = lk[x][i];
                out_idx[o + i] = li[x][i];
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// 1'''. Shortlist on v_mfma_f32_16x16x32_f16.  Under load the chip holds a higher clock on the
// 16x16x32 shape than on 32x32x16 at equal cycles per flop (MI355X_MICROARCH.md, DVFS item 7), so the
// D=192 hot path runs on it.  16-row fragment layout (prep16_kernel): lane l of block b holds row
// b*16 + (l & 15), k = s*32 + 8*(l >> 4) + j; the accumulator of lane l holds rows 4*(l >> 4) + i of
// query column l & 15, i.e. each query's candidates are spread over 4 lanes (lane groups g = 0..3), and
// perm16 puts the 4 mirror candidates of a tile into 4 different groups.  Wave = QB query blocks of 16.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int perm16(int r) { return ((r & 3) << 2) | (r >> 2); }

struct Prep16Args {
    const float *rows;
    long n;
    int d, S;       // S = k-steps of 32
    float scale;
    half8 *frag;    // [ceil(n/16)][S][64][8]
    float *seed;    // dataset: [ceil(n/16)][16] -||c||^2/2 by A row (-inf on padding rows); queries: null
    int perm;
    int dcfirst;    // 1 (d = 192, both operands alike): the three PsyV DC dimensions 0, 64, 128 in k-step 0
};

// Fragment position k -> descriptor dimension.  A flat tile's Haar PsyV (one colour) is exactly zero but in the Y, U
// and V DC (dimensions 0, 64, 128); swapping 64 <-> 1 and 128 <-> 2 on BOTH sides (the contraction is invariant under
// a common permutation) puts all three into k-step 0, so a workgroup of flat queries needs k-step 0 only: the other
// k-steps would add exactly +-0 products to every accumulator.
__device__ __forceinline__ int dc_first_dim(int k) {
    return k == 1 ? 64 : k == 64 ? 1 : k == 2 ? 128 : k == 128 ? 2 : k;
}

__global__ __launch_bounds__(256) void prep16_kernel(Prep16Args a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
    const long nblk = (a.n + 15) / 16;
    for (long blk = (long)blockIdx.x * 4 + wave; blk < nblk; blk += (long)gridDim.x * 4) {
        const long row = blk * 16 + (a.perm ? perm16(r) : r);
        const bool valid = row < a.n;
        double s2 = 0;
        const bool vec = (a.d & 7) == 0 && (((uintptr_t)a.rows) & 31) == 0;
        for (int s = 0; s < a.S; s++) {
            half8 hv;
            float vv[8];
            const int k0 = s * 32 + 8 * g;
            if (vec) {  // the piece's 8 consecutive dimensions in two 16-byte loads, then the DC swaps of dc_first_dim
                float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
                if (valid && k0 < a.d) {
                    const float4 *src = reinterpret_cast<const float4 *>(a.rows + row * a.d + k0);
                    x0 = src[0];
                    x1 = src[1];
                }
                vv[0] = x0.x; vv[1] = x0.y; vv[2] = x0.z; vv[3] = x0.w;
                vv[4] = x1.x; vv[5] = x1.y; vv[6] = x1.z; vv[7] = x1.w;
                if (a.dcfirst && valid && (k0 == 0 || k0 == 64 || k0 == 128) && k0 < a.d) {
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const int kd = dc_first_dim(k0 + j);
                        if (kd != k0 + j) vv[j] = a.rows[row * a.d + kd];
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int k = k0 + j;
                    const int kd = a.dcfirst ? dc_first_dim(k) : k;
                    vv[j] = (valid && k < a.d) ? a.rows[row * a.d + kd] : 0.0f;
                }
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float v = vv[j];
                const float vs = v * a.scale;
                _Float16 vh = (_Float16)vs;
                if (fabsf((float)vh) < 6.103515625e-05f) vh = (_Float16)0.0f;  // as prep_rows_kernel
                hv[j] = vh;
                s2 += (double)vs * (double)vs;
            }
            a.frag[(blk * a.S + s) * 64 + lane] = hv;
        }
        if (a.seed) {
            s2 += __shfl_xor(s2, 16, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (g == 0) a.seed[blk * 16 + r] = valid ? -0.5f * (float)s2 : -INFINITY;
        }
    }
}

// FLAT: a workgroup whose queries are all flat tiles (grouped last by nn_frame_tiling_dev; their fragments are zero
// beyond k-step 0, dc_first_dim): per candidate block only k-step 0 is streamed (1 of S KB) and contracted, the
// same keys bit for bit.
// MODE (timing experiments of the experiment build only; results invalid when != 0): 1 no list insertion, 2 no
// epilogue, 3 no epilogue and no A-fragment reads inside the stage (the MFMA + stream floor)
template <int N>
__device__ __forceinline__ void vm_wait() {  // s_waitcnt vmcnt(N): all but this wave's N youngest vector-memory ops
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// VAR bit 0: per query block, a wave-uniform test before its 4 per-element list tests, thresholds kept in registers
// (the same comparisons, so the same lists); bit 1: a 3-buffer LDS ring (two stages in flight instead of one).
// Measured and removed (round 5, DESIGN.md section 4, identical digests): a software-pipelined stage (block cb + 1's
// MFMAs before block cb's epilogue, one compare per element) +1.5..3 %; 4 blocks per stage +1..3 %; 4 blocks per
// stage with the insertions queued per lane in LDS and applied in bulk +6 % (commit c152f52 has both).
// gate (VAR bit 0 only; nullptr: off): the k = 1 search's exact insertion gate (round 6).  The rescore needs every
// candidate whose key can reach T(kk), kk the smallest key of the query (nn_rescore_kernel; T increasing in kk), and
// T(kk) <= T(b) for every key b the query has already seen.  So a lane may skip any candidate whose key exceeds
// T(best key of the query so far, over its 4 lanes): gate[q] = (x, y) with T(b) <= (b + x) * gb + y up to the
// fp32 slack added here (gate16_kernel).  Each lane's own L-th key still gates its list as before; the tighter of the
// two is kept current in th[] whenever the wave takes the insertion branch (the 4 lanes' bests by two xor shuffles).
// A lane's list keeps every candidate the rescore can need, so the overflow rule and tiers 2 / 3 are unchanged.
template <int S, int L, int CB, int NW, int QB, bool FLAT, int MODE = 0, int VAR = 0>
__device__ __forceinline__ void shortlist16_body(const half8 *__restrict__ cfrag, const float *__restrict__ cseed,
                                                 int nblk, const half8 *__restrict__ qfrag, int nq, int blk_per_split,
                                                 int nsplit, int perm, float *__restrict__ out_key,
                                                 int *__restrict__ out_idx, const float2 *__restrict__ gate,
                                                 float gb) {
    typedef float floatx4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int FRAG_BYTES = CB * S * 1024;
    constexpr int BUF_BYTES = FRAG_BYTES + CB * 64;
    constexpr int NT = NW * 64;
    constexpr int PER_T = CB * S * 64 / NT;
    static_assert((CB * S * 64) % NT == 0 && S % 2 == 0, "stage must split evenly over the workgroup");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const int nqblk = (nq + 15) / 16;
    const int qb0 = (blockIdx.x * NW + w) * QB;
    const int split = blockIdx.y;
    const int b_begin = split * blk_per_split;
    const int b_end = min(nblk, b_begin + blk_per_split);

    half8 bq[QB][S];
#pragma unroll
    for (int q = 0; q < QB; q++) {
        const long qq = min(qb0 + q, nqblk - 1);  // blocks past the end: clamped duplicate, never written
#pragma unroll
        for (int s = 0; s < S; s++) bq[q][s] = qfrag[(qq * S + s) * 64 + lane];
    }
    // land the query fragments before the loop (a real s_waitcnt the compiler's pass accounts for): a
    // wait sunk into the loop would also count the hidden LDS-DMA pieces and stall on them
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    float lk[QB][L];
    int li[QB][L];
#pragma unroll
    for (int q = 0; q < QB; q++)
#pragma unroll
        for (int i = 0; i < L; i++) {
            lk[q][i] = INFINITY;
            li[q][i] = -1;
        }
    // candidate index of accumulator element i of this lane, relative to the block
    int rel[4];
#pragma unroll
    for (int i = 0; i < 4; i++) rel[i] = perm ? perm16(4 * g + i) : 4 * g + i;

    const int nstage = (b_end > b_begin) ? (b_end - b_begin + CB - 1) / CB : 0;
    auto issue = [&](int st, int buf) {
        const int blk0 = b_begin + st * CB;
        const int nb = min(CB, b_end - blk0);
        const uint4 *src = reinterpret_cast<const uint4 *>(cfrag) + (long)blk0 * S * 64 + w * 64 + lane;
        char *dst = smem + buf * BUF_BYTES + w * 1024;
        if constexpr (FLAT) {  // wave w: k-step 0 of block w (the last block again past the end: never read)
            static_assert(CB <= NW, "one k-step-0 piece per wave");
            if (CB == NW || w < CB)
                glds16_asm(reinterpret_cast<const uint4 *>(cfrag) + (long)(blk0 + min(w, nb - 1)) * S * 64 + lane,
                           smem + buf * BUF_BYTES + w * S * 1024);
        } else if (nb == CB) {
#pragma unroll
            for (int j = 0; j < PER_T; j++) glds16_asm(src + j * NT, dst + j * NT * 16);
        } else {
            const int last = nb * S * 64 - 1 - (w * 64 + lane);
#pragma unroll
            for (int j = 0; j < PER_T; j++) glds16_asm(src + min(j * NT, last), dst + j * NT * 16);
        }
        if (w == 0 && lane < CB * 4)
            glds16_asm(reinterpret_cast<const uint4 *>(cseed) + (long)blk0 * 4 + min(lane, nb * 4 - 1),
                       smem + buf * BUF_BYTES + FRAG_BYTES);
    };

    constexpr int NBUF = (VAR & 2) ? 3 : 2;
    // a stage's DMA instructions per wave (the seed piece is wave 0's): the counted wait of the 3-buffer ring
    auto wait_all_but_next = [&]() {
        if (w == 0) vm_wait<(FLAT ? 1 : PER_T) + 1>();
        else vm_wait<(FLAT ? 1 : PER_T)>();
    };
    float th[QB];  // VAR & 1: max(-0.5 * lk[q][L - 1], the gate's bound), kept current
    float2 gq[QB];  // the gate of this lane's query of block q (x = +inf: none)
#pragma unroll
    for (int q = 0; q < QB; q++) {
        th[q] = -INFINITY;
        const int qq = (qb0 + q) * 16 + (lane & 15);
        gq[q] = (gate && qq < nq) ? gate[qq] : make_float2(INFINITY, INFINITY);
    }
    if (nstage > 0) issue(0, 0);
    if (NBUF == 3 && nstage > 1) {
        issue(1, 1);
        wait_all_but_next();
    } else {
        dma_drain();
    }
    __syncthreads();
    for (int st = 0; st < nstage; st++) {
        const char *B = smem + (st % NBUF) * BUF_BYTES;
        const half8 *A = reinterpret_cast<const half8 *>(B) + lane;
        const floatx4 *SD = reinterpret_cast<const floatx4 *>(B + FRAG_BYTES) + g;
        floatx4 sd[CB];
#pragma unroll
        for (int cb = 0; cb < CB; cb++) sd[cb] = SD[cb * 4];
        half8 a0 = A[0], a1 = A[64];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (st + NBUF - 1 < nstage) issue(st + NBUF - 1, (st + NBUF - 1) % NBUF);
#pragma unroll
        for (int cb = 0; cb < CB; cb++) {
            const int blk = b_begin + st * CB + cb;
            if (blk < b_end) {
                floatx4 acc[QB];
                if constexpr (FLAT) {
                    const half8 af = A[(cb * S) * 64];
#pragma unroll
                    for (int q = 0; q < QB; q++)
                        acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bq[q][0], sd[cb], 0, 0, 0);
                } else {
#pragma unroll
                for (int s = 0; s < S; s += 2) {
                    half8 n0, n1;
                    const bool more = MODE != 3 && (s + 2 < S || cb + 1 < CB);
                    if constexpr (MODE == 3) {
                    } else if (s + 2 < S) {
                        n0 = A[(cb * S + s + 2) * 64];
                        n1 = A[(cb * S + s + 3) * 64];
                    } else if (cb + 1 < CB) {
                        n0 = A[((cb + 1) * S) * 64];
                        n1 = A[((cb + 1) * S + 1) * 64];
                    }
#pragma unroll
                    for (int q = 0; q < QB; q++)
                        acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bq[q][s], s == 0 ? sd[cb] : acc[q], 0, 0, 0);
#pragma unroll
                    for (int q = 0; q < QB; q++)
                        acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bq[q][s + 1], acc[q], 0, 0, 0);
                    if (more) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2 * QB, 0);
                    if (more) {
                        a0 = n0;
                        a1 = n1;
                    }
                }
                }
                if constexpr (MODE >= 2) {
#pragma unroll
                    for (int q = 0; q < QB; q++) li[q][0] += __float_as_int(acc[q][0]) & 1;  // keeps the MFMAs live
                    continue;
                }
                // epilogue: acc = q.c - ||c||^2/2, key = -2 acc; one wave-uniform branch per block
                bool need = false;
                float m[QB];
#pragma unroll
                for (int q = 0; q < QB; q++) {
                    m[q] = fmaxf(fmaxf(acc[q][0], acc[q][1]), fmaxf(acc[q][2], acc[q][3]));
                    need |= m[q] > ((VAR & 1) ? th[q] : -0.5f * lk[q][L - 1]);
                }
                if constexpr (MODE == 1) {
                    li[0][0] += need ? 1 : 0;
                    continue;
                }
                if (__builtin_expect(__any(need), 0)) {
                    const int base = blk * 16;
                    if constexpr ((VAR & 1) != 0) {
#pragma unroll
                        for (int q = 0; q < QB; q++)
                            if (__any(m[q] > th[q]))
#pragma unroll
                                for (int i = 0; i < 4; i++)
                                    if (acc[q][i] > th[q]) {
                                        list_insert<L>(lk[q], li[q], -2.0f * acc[q][i], base + rel[i]);
                                        th[q] = fmaxf(th[q], -0.5f * lk[q][L - 1]);
                                    }
                        if (gate) {  // wave-uniform: the query's best key over its 4 lanes -> its gate
#pragma unroll
                            for (int q = 0; q < QB; q++) {
                                float b = lk[q][0];
                                b = fminf(b, __shfl_xor(b, 16, 64));
                                b = fminf(b, __shfl_xor(b, 32, 64));
                                if (gq[q].x < INFINITY && b < INFINITY) {
                                    const float X = b + gq[q].x, T1 = X * gb, T2 = T1 + gq[q].y;
                                    // every rounding of the three ops, and the rescore's 1e-12 |kk| term, inside
                                    const float T = T2 + (fabsf(T1) + fabsf(gq[q].y)) * 9.5367431640625e-07f + 1e-30f;
                                    th[q] = fmaxf(th[q], -0.5f * T);
                                }
                            }
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < QB; q++)
#pragma unroll
                            for (int i = 0; i < 4; i++)
                                if (acc[q][i] > -0.5f * lk[q][L - 1])
                                    list_insert<L>(lk[q], li[q], -2.0f * acc[q][i], base + rel[i]);
                    }
                }
            }
        }
        if (NBUF == 3 && st + 2 < nstage)
            wait_all_but_next();  // stage st + 1 landed, st + 2 may still be in flight
        else
            dma_drain();
        __syncthreads();
    }
    // partial lists: [q][split][g][L]
#pragma unroll
    for (int q = 0; q < QB; q++) {
        const int qq = (qb0 + q) * 16 + (lane & 15);
        if (qq < nq) {
            const long o = (((long)qq * nsplit + split) * 4 + g) * L;
#pragma unroll
            for (int i = 0; i < L; i++) {
                out_key[o + i] = lk[q][i];
                out_idx[o + i] = li[q][i];
            }
        }
    }
}

// flat_cnt (or null): device count of the batch's non-flat queries, the flat ones placed after them
template <int S, int L, int CB, int NW, int QB, int MODE = 0, int VAR = 0>
__global__ __launch_bounds__(NW * 64, 1) void nn_shortlist16_kernel(const half8 *__restrict__ cfrag,
                                                                const float *__restrict__ cseed, int nblk,
                                                                const half8 *__restrict__ qfrag, int nq,
                                                                int blk_per_split, int nsplit, int perm,
                                                                float *__restrict__ out_key,
                                                                int *__restrict__ out_idx, const int *flat_cnt,
                                                                const float2 *__restrict__ gate, float gb) {
    if (flat_cnt && (long)blockIdx.x * (NW * QB * 16) >= (long)*flat_cnt)
        shortlist16_body<S, L, CB, NW, QB, true, MODE, VAR>(cfrag, cseed, nblk, qfrag, nq, blk_per_split, nsplit, perm,
                                                            out_key, out_idx, gate, gb);
    else
        shortlist16_body<S, L, CB, NW, QB, false, MODE, VAR>(cfrag, cseed, nblk, qfrag, nq, blk_per_split, nsplit,
                                                             perm, out_key, out_idx, gate, gb);
}

// The k = 1 gate of nn_shortlist16_kernel: T(kk) <= (kk + x) * gb + y for the rescore's threshold
//     T(kk) = (n2 + kk + Ek)(1 + g)/(1 - g) - n2 + Ek + 1e-12 (n2 + |kk|) + 1e-30     (nn_rescore_kernel)
// x = n2 + Ek and y = -n2 + Ek + 1e-12 n2 + 1e-30 rounded up to fp32, gb = (1 + g)/(1 - g) rounded up (host); the
// kernel's fp32 slack covers its own roundings and the 1e-12 |kk| term.  Queries the rescore sends to tier 3: no gate.
__global__ __launch_bounds__(256) void gate16_kernel(const QStat *__restrict__ qs, int nq, int d, double N, double H,
                                                     double Ec, float2 *__restrict__ gate) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    const QStat st = qs[q];
    if (st.flags & QF_BAD) {
        gate[q] = make_float2(INFINITY, INFINITY);
        return;
    }
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double gam = 2.0 * (d + 1) * u;
    const double Ek = 1.05 * (2.0 * u * N * N + gam * (N * N + 2.0 * st.hn * H) + 2.0 * (st.en * N + st.hn * Ec)) + 1e-30;
    const double x = st.n2 + Ek, y = -st.n2 + Ek + 1e-12 * st.n2 + 1e-30;
    float xf = (float)x, yf = (float)y;
    if ((double)xf < x) xf = nextafterf(xf, INFINITY);
    if ((double)yf < y) yf = nextafterf(yf, INFINITY);
    gate[q] = make_float2(xf, yf);
}

// ------------------------------------------------------------------------------------------
// 1b. tier-2 collect: for the queries whose tier-1 lists overflowed, recompute the MFMA keys and append
// EVERY candidate with key <= T(q) to a per-query buffer (atomic cursor).  Compact query j's B fragment
// is gathered straight from the tier-1 fragment buffer.  Grid-stride over groups of 256 queries.
// ------------------------------------------------------------------------------------------
template <int S, int CB>
__global__ __launch_bounds__(256, 2) void nn_collect_kernel(const half8 *__restrict__ cfrag,
                                                            const float *__restrict__ cnc, int nblk,
                                                            const half8 *__restrict__ qfrag, const int *fb_list,
                                                            const int *fb_count, int jbase, int chunk,
                                                            const float *thr, int blk_per_split, int perm, int *ccnt,
                                                            int *cbuf, int cap) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int FRAG_BYTES = CB * S * 1024;
    constexpr int BUF_BYTES = FRAG_BYTES + CB * 128;
    constexpr int PER_T = CB * S * 64 / 256;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int count = min(*fb_count - jbase, chunk);  // this chunk's slots (local index j = slot - jbase)
    const int b_begin = blockIdx.y * blk_per_split;
    const int b_end = min(nblk, b_begin + blk_per_split);
    const half8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
    fb_list += jbase;
    for (int g = blockIdx.x; g * 256 < count; g += gridDim.x) {
        half8 bq0[S], bq1[S];
        int j0 = (g * 4 + w) * 64 + (lane & 31), j1 = j0 + 32;
        const int q0 = j0 < count ? fb_list[j0] : -1, q1 = j1 < count ? fb_list[j1] : -1;
        const float t0 = q0 >= 0 ? thr[q0] : -INFINITY, t1 = q1 >= 0 ? thr[q1] : -INFINITY;
#pragma unroll
        for (int s = 0; s < S; s++) {
            bq0[s] = q0 >= 0 ? qfrag[((long)(q0 >> 5) * S + s) * 64 + (q0 & 31) + 32 * h] : zero8;
            bq1[s] = q1 >= 0 ? qfrag[((long)(q1 >> 5) * S + s) * 64 + (q1 & 31) + 32 * h] : zero8;
        }
        const int nstage = (b_end > b_begin) ? (b_end - b_begin + CB - 1) / CB : 0;
        uint4 stg[PER_T];
        uint4 stg_nc = make_uint4(0, 0, 0, 0);
        auto gload = [&](int st) {
            const int blk0 = b_begin + st * CB;
            const int last = min(CB, b_end - blk0) * S * 64 - 1;
            const uint4 *src = reinterpret_cast<const uint4 *>(cfrag) + (long)blk0 * S * 64;
#pragma unroll
            for (int jj = 0; jj < PER_T; jj++) stg[jj] = src[min(tid + jj * 256, last)];
            stg_nc = reinterpret_cast<const uint4 *>(cnc)[(long)blk0 * 8 + min(tid, min(CB, b_end - blk0) * 8 - 1)];
        };
        auto swrite = [&](int buf) {
            uint4 *dst = reinterpret_cast<uint4 *>(smem + buf * BUF_BYTES);
#pragma unroll
            for (int jj = 0; jj < PER_T; jj++) dst[tid + jj * 256] = stg[jj];
            if (tid < CB * 8) reinterpret_cast<uint4 *>(smem + buf * BUF_BYTES + FRAG_BYTES)[tid] = stg_nc;
        };
        __syncthreads();
        if (nstage > 0) {
            gload(0);
            swrite(0);
        }
        __syncthreads();
        for (int st = 0; st < nstage; st++) {
            if (st + 1 < nstage) gload(st + 1);
            const char *B = smem + (st & 1) * BUF_BYTES;
            for (int cb = 0; cb < CB; cb++) {
                const int blk = b_begin + st * CB + cb;
                if (blk >= b_end) break;
                floatx16 acc0 = {0}, acc1 = {0};
#pragma unroll
                for (int s = 0; s < S; s++) {
                    const half8 av = reinterpret_cast<const half8 *>(B)[(cb * S + s) * 64 + lane];
                    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq0[s], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq1[s], acc1, 0, 0, 0);
                }
                const float *np = reinterpret_cast<const float *>(B + FRAG_BYTES) + cb * 32 + h * 16;
                // one slot reservation per lane and block (not one returning atomic per candidate)
                unsigned m0 = 0, m1 = 0;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const float nc = np[r];
                    m0 |= (fmaf(-2.0f, acc0[r], nc) <= t0) ? 1u << r : 0u;
                    m1 |= (fmaf(-2.0f, acc1[r], nc) <= t1) ? 1u << r : 0u;
                }
                int p0 = m0 ? atomicAdd(&ccnt[j0], __popc(m0)) : 0;
                int p1 = m1 ? atomicAdd(&ccnt[j1], __popc(m1)) : 0;
                while (m0 | m1) {
                    if (m0) {
                        const int r = __ffs(m0) - 1, row = (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (p0 < cap) cbuf[(long)j0 * cap + p0] = blk * 32 + (perm ? row_perm(row) : row);
                        p0++;
                        m0 &= m0 - 1;
                    }
                    if (m1) {
                        const int r = __ffs(m1) - 1, row = (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (p1 < cap) cbuf[(long)j1 * cap + p1] = blk * 32 + (perm ? row_perm(row) : row);
                        p1++;
                        m1 &= m1 - 1;
                    }
                }
            }
            if (st + 1 < nstage) swrite((st + 1) & 1);
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------------
// 2. rescore: one wave per query.
// ------------------------------------------------------------------------------------------
struct RescoreArgs {
    const float *rows;   // [n][d]
    const float *q;      // [nq][d]
    const QStat *qstat;
    const float *key;
    const int *idx;
    int n, d, nq, k, L, nsplit;
    int lpq;             // lanes (partial lists) per query and split: 2 (32x32 shortlist) or 4 (16x16)
    double N, H, Ec, max_abs_c;
    int ds_int;
    int *out_idx;
    float *out_err;
    int *fb_list;        // tier 2: overflowed queries (MFMA collect pass), count in fb_count
    int *fb_count;
    float *thr;          // [nq] tier-2 threshold T (rounded up to fp32)
    int *ex_list;        // tier 3: exhaustive scan (bad queries, collect-buffer overflow)
    int *ex_count;
    int *ccnt;           // [fb_max] collected candidates per tier-2 query
    int *cbuf;           // [fb_max][cap]
    int cap, fb_max;
    const int32_t *tr_tile, *tr_pal;
    const uint8_t *tr_attr;
    int32_t *m_tile, *m_pal;
    uint8_t *m_hm, *m_vm;
    const KdOrder *ko;   // tie order: ANN's kd-tree first-found (device view) or nullptr = the lowest index
    int *kd_list, *kd_count;  // (unused by the small-batch scan since round 5: its merge replays in place)
    int force_replay;         // test hook (tiler_debug_force_replay): the check vouches for nothing
    int prune;                // small-batch scan with a kd-tree of > bs points: the merge kernel runs ANN's pruning
                              // check (kd_verify_kernel's test) and replays a query it cannot vouch for itself
    int *h_idx;               // small-batch scan: host-visible copies of the final results (null: none)
    float *h_err;
};

__device__ __forceinline__ void write_map(const RescoreArgs &a, long q, int best) {
    if (!a.m_tile) return;
    a.m_tile[q] = best >= 0 ? a.tr_tile[best] : -1;
    a.m_pal[q] = best >= 0 ? a.tr_pal[best] : -1;
    const int at = best >= 0 ? a.tr_attr[best] : 0;
    a.m_hm[q] = (at & 1) != 0;
    a.m_vm[q] = (at & 2) != 0;
}

// any() over this lane's group of W lanes (W divides 64)
template <int W>
__device__ __forceinline__ bool grp_any(bool p) {
    const unsigned long long b = __ballot(p);
    if constexpr (W == 64) {
        return b != 0;
    } else {
        const int g = (int)(threadIdx.x & 63) / W;
        return ((b >> (g * W)) & ((1ull << W) - 1)) != 0;
    }
}

// lexicographic (v, i) minimum over a group of W lanes
template <int W>
__device__ __forceinline__ void grp_argmin(float &v, int &i) {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        const bool take = (ov < v) || (ov == v && (unsigned)oi < (unsigned)i);
        v = take ? ov : v;
        i = take ? oi : i;
    }
}

// W lanes per query: 64 (one wave), or 16 when the query has at most 16 list entries (the 16x16x32 shortlist with
// one split: 4 lanes x L = 4), four queries per wave -- the entries' exact distances (192 dependent fp32 adds
// each) then fill the wave instead of a quarter of it
template <int W>
__global__ __launch_bounds__(256) void nn_rescore_kernel(RescoreArgs a) {
    const int lane = threadIdx.x & (W - 1);
    const long q = (long)blockIdx.x * (256 / W) + (threadIdx.x / W);
    if (q >= a.nq) return;  // whole groups
    const int E = a.nsplit * a.lpq * a.L;  // list entries per query
    float key = INFINITY;
    int idx = -1;
    if (lane < E) {
        key = a.key[q * E + lane];
        idx = a.idx[q * E + lane];
    }
    const QStat st = a.qstat[q];
    if (st.flags & QF_BAD) {  // fp16 overflow / non-finite: no valid MFMA keys -> exhaustive scan
        if (lane == 0) a.ex_list[atomicAdd(a.ex_count, 1)] = (int)q;
        return;
    }
    bool fallback = false;
    // k-th smallest key (lexicographic by (key, lane) so duplicates count separately)
    float kk = INFINITY;
    {
        float v = (idx >= 0) ? key : INFINITY;
        int who = lane;
        bool taken = false;
        for (int r = 0; r < a.k; r++) {
            float mv = taken ? INFINITY : v;
            int mi = taken ? 0x7fffffff : who;
            grp_argmin<W>(mv, mi);
            kk = mv;
            if (lane == mi) taken = true;
        }
    }
    // threshold T (DESIGN.md "Exactness argument")
    double T;
    const double u = 5.9604644775390625e-08;  // 2^-24
    const bool exact = a.ds_int && (st.flags & QF_INT) &&
                       (double)a.d * a.max_abs_c * (double)st.pad * 4.0 < 16777216.0 &&
                       (double)a.d * a.max_abs_c * a.max_abs_c < 16777216.0;
    if (exact) {
        T = kk;
    } else {
        const double nq = sqrt(st.n2);
        // key error bound: fp32 rounding of ||c||^2, the MFMA accumulation seeded with
        // -||c||^2/2 (>= 2x gamma_{D+1} over |seed| + sum |q^_d c^_d|), and the fp16 residuals
        const double gam = 2.0 * (a.d + 1) * u;
        const double Ek = 1.05 * (2.0 * u * a.N * a.N + gam * (a.N * a.N + 2.0 * st.hn * a.H) +
                                  2.0 * (st.en * a.N + st.hn * a.Ec)) + 1e-30;
        const double g = (double)(a.d + 4) * u / (1.0 - (double)(a.d + 4) * u) * 1.05;
        T = ((st.n2 + (double)kk + Ek) * (1.0 + g) / (1.0 - g)) - st.n2 + Ek;
        T += 1e-12 * (st.n2 + fabs((double)kk)) + 1e-30;
        (void)nq;
    }
    if (!isfinite(kk)) T = INFINITY;
    // overflow: a full list whose last kept key is <= T may have dropped a needed candidate.  Exact integer keys
    // with L >= k need no check under index order (a lane keeps its best L by (key, index), consistent with the
    // global order), but under ANN's kd order a lane's dropped equal-key entry can rank first
    if (!exact || a.L < a.k || a.ko) {
        const bool last = lane < E && (lane % a.L) == a.L - 1;
        if (grp_any<W>(last && idx >= 0 && (double)key <= T)) fallback = true;
    }
    const bool cand = (idx >= 0) && ((double)key <= T);
    float dist = INFINITY;
    int di = 0x7fffffff;
    if (!fallback && cand) {
        dist = exact_dist(a.q + q * a.d, a.rows + (long)idx * a.d, a.d);
        di = idx;
    }
    if (fallback) {
        if (lane == 0) {
            float tf = (float)T;
            if ((double)tf < T) tf = nextafterf(tf, INFINITY);  // keep T an upper bound in fp32
            a.thr[q] = tf;
            const int p = atomicAdd(a.fb_count, 1);
            if (p < a.fb_max)
                a.fb_list[p] = (int)q;
            else
                a.ex_list[atomicAdd(a.ex_count, 1)] = (int)q;
        }
        return;
    }
    // top-k by (dist, tie order)
    const float *qrow = a.q + q * a.d;
    bool taken = false;
    for (int r = 0; r < a.k; r++) {
        float mv = taken ? INFINITY : dist;
        int mi = taken ? 0x7fffffff : di;
        kd_argmin<W>(a.ko, qrow, mv, mi);
        if (!taken && di == mi && mi != 0x7fffffff) taken = true;
        if (lane == 0) {
            const bool ok = mi != 0x7fffffff;
            a.out_idx[q * a.k + r] = ok ? mi : -1;
            a.out_err[q * a.k + r] = ok ? mv : FLT_MAX;
            if (r == 0) write_map(a, q, ok ? mi : -1);
        }
    }
}

// ------------------------------------------------------------------------------------------
// 2b. tier-2 rescore: every collected candidate (key <= T) rescored exactly; top-k by (dist, index).
// One wave per compact query; a buffer that overflowed its capacity sends the query to tier 3.
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void nn_rescore2_kernel(RescoreArgs a, int jbase, int chunk) {
    const int lane = threadIdx.x & 63;
    const int count = min(*a.fb_count - jbase, chunk);
    for (long j = (long)blockIdx.x * 4 + (threadIdx.x >> 6); j < count; j += (long)gridDim.x * 4) {
        const long q = a.fb_list[jbase + j];
        int n = 0;
        if (lane == 0) n = atomicExch(a.ccnt + j, 0);  // read and clean for the next chunk
        n = __shfl(n, 0, 64);
        if (n > a.cap) {
            if (lane == 0) a.ex_list[atomicAdd(a.ex_count, 1)] = (int)q;
            continue;
        }
        float bd[8];
        int bi[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            bd[i] = INFINITY;
            bi[i] = 0x7fffffff;
        }
        const float *qrow = a.q + q * a.d;
        for (int e = lane; e < n; e += 64) {
            const int idx = a.cbuf[j * a.cap + e];
            const float dist = exact_dist(qrow, a.rows + (long)idx * a.d, a.d);
            if (!kd_less(a.ko, qrow, dist, idx, bd[7], bi[7])) continue;
            kd_list_insert<8>(a.ko, qrow, bd, bi, dist, idx);  // (dist, tie order); entries arrive in no order
        }
        int ptr = 0;
        for (int r = 0; r < a.k; r++) {
            float hv = INFINITY;
            int hi = 0x7fffffff;
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i == ptr) {
                    hv = bd[i];
                    hi = bi[i];
                }
            float mv = hv;
            int mi = hi;
            kd_argmin<64>(a.ko, qrow, mv, mi);
            if (hi == mi && mi != 0x7fffffff) ptr++;
            if (lane == 0) {
                const bool ok = mi != 0x7fffffff;
                a.out_idx[q * a.k + r] = ok ? mi : -1;
                a.out_err[q * a.k + r] = ok ? mv : FLT_MAX;
                if (r == 0) write_map(a, q, ok ? mi : -1);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// 3. exhaustive exact scan (queued queries, k > 8): one workgroup per query, grid-stride list.
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void nn_exact_kernel(RescoreArgs a, int list_n) {
    __shared__ float sq[1024];
    __shared__ float sd[256 * K];
    __shared__ int si[256 * K];
    const int tid = threadIdx.x;
    const int count = a.ex_list ? *a.ex_count : list_n;
    for (int qi = blockIdx.x; qi < count; qi += gridDim.x) {
        const long q = a.ex_list ? a.ex_list[qi] : qi;
        __syncthreads();
        for (int i = tid; i < a.d; i += 256) sq[i] = a.q[q * a.d + i];
        __syncthreads();
        float bd[K];
        int bi[K];
#pragma unroll
        for (int i = 0; i < K; i++) {
            bd[i] = FLT_MAX;
            bi[i] = -1;
        }
        int cnt = 0;
        for (int j = tid; j < a.n; j += 256) {
            const float *c = a.rows + (long)j * a.d;
            float dist = 0.0f;
            const float lim = (cnt < K) ? INFINITY : bd[K - 1];
            int i = 0;
            for (; i < a.d; i++) {
                const float t = sq[i] - c[i];
                dist = dist + t * t;
                if (dist > lim) break;
            }
            if (i < a.d) continue;
            if (cnt == K && !kd_less(a.ko, sq, dist, j, bd[K - 1], bi[K - 1])) continue;
            if (!a.ko)
                list_insert<K>(bd, bi, dist, j);  // j ascends: an equal key stays behind, as index order wants
            else
                kd_list_insert<K>(a.ko, sq, bd, bi, dist, j, cnt < K ? cnt : K - 1);
            if (cnt < K) cnt++;
        }
#pragma unroll
        for (int i = 0; i < K; i++) {
            sd[tid * K + i] = (i < cnt) ? bd[i] : INFINITY;
            si[tid * K + i] = (i < cnt) ? bi[i] : 0x7fffffff;
        }
        __syncthreads();
        if (tid < 64) {
            // each lane holds 4 thread lists; extract the k best by (dist, idx)
            int ptr[4] = {0, 0, 0, 0};
            for (int r = 0; r < a.k; r++) {
                float lv = INFINITY;
                int li = 0x7fffffff, lt = -1;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int th = tid * 4 + t;
                    if (ptr[t] < K) {
                        const float v = sd[th * K + ptr[t]];
                        const int ii = si[th * K + ptr[t]];
                        if (kd_less(a.ko, sq, v, ii, lv, li)) {
                            lv = v;
                            li = ii;
                            lt = t;
                        }
                    }
                }
                float mv = lv;
                int mi = li;
                kd_argmin<64>(a.ko, sq, mv, mi);
                if (lt >= 0 && li == mi && mi != 0x7fffffff) ptr[lt]++;
                if (tid == 0) {
                    const bool ok = mi != 0x7fffffff;
                    a.out_idx[q * a.k + r] = ok ? mi : -1;
                    a.out_err[q * a.k + r] = ok ? mv : FLT_MAX;
                    if (r == 0) write_map(a, q, ok ? mi : -1);
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// 4. small batches (the reference's per-tile calls: ann_kdtree_search per frame tile, main.pas:4027, coalesced by the
// library into batches of a few queries): an exhaustive exact scan spread over the whole GPU.  Grid = candidate
// splits; each workgroup scans its contiguous candidate range for ALL the batch's queries (staged in LDS), one
// candidate per thread at a time, each query's fp32 distance summed in dimension order (the reference's sequential
// sum), the K best per (thread, query) by (distance, tie order); then the workgroup's K best per query -> partials
// [q][split][K].  nn_scan_merge_kernel picks the k best of each query's partials.  No MFMA, no tiers: the shortlist's
// fixed costs (a 512-query workgroup per split, fragment prep, rescore) dominated a call of one query (0.6 ms).
// ------------------------------------------------------------------------------------------
static constexpr int SCAN_D_MAX = 256;
// One term of the reference's sequential sum, d + (q - c)^2 rounded after the product and after the sum (the mode's
// IEEE single ops, as the compiler's own).  Written as one asm block so that the vectoriser cannot pack the
// independent per-query sums into v_pk_add_f32 / v_pk_mul_f32 with v_mov shuffles (measured slower here).
__device__ __forceinline__ float sq_acc(float d, float q, float c) {
    float t;
    asm("v_sub_f32 %1, %2, %3\n\tv_mul_f32 %1, %1, %1\n\tv_add_f32 %0, %0, %1" : "+v"(d), "=&v"(t) : "v"(q), "v"(c));
    return d;
}
template <int QN, int K>
__global__ __launch_bounds__(256) void nn_scan_small_kernel(RescoreArgs a, int nsplit, float *__restrict__ pd,
                                                            int *__restrict__ pi) {
    __shared__ __attribute__((aligned(16))) float sq[QN * SCAN_D_MAX];
    __shared__ float rd[4][K];
    __shared__ int ri[4][K];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int qg = blockIdx.y * QN;  // this workgroup's group of queries
    const int nq = min(a.nq - qg, QN), d = a.d;
    for (int i = tid; i < nq * d; i += 256)
        sq[(i / d) * SCAN_D_MAX + i % d] = a.q[(long)(qg + i / d) * d + i % d];
    __syncthreads();
    const long c0 = (long)a.n * blockIdx.x / nsplit, c1 = (long)a.n * (blockIdx.x + 1) / nsplit;
    float bd[QN][K];
    int bi[QN][K];
#pragma unroll
    for (int q = 0; q < QN; q++)
#pragma unroll
        for (int r = 0; r < K; r++) {
            bd[q][r] = INFINITY;
            bi[q][r] = 0x7fffffff;
        }
    for (long j = c0 + tid; j < c1; j += 256) {
        const float *c = a.rows + j * d;
        float dist[QN];
#pragma unroll
        for (int q = 0; q < QN; q++) dist[q] = 0.0f;
        if constexpr (QN == 1) {  // one sum per row: the compiler keeps 8 loads in flight by itself
            for (int d0 = 0; d0 < d; d0 += 4) {  // d % 4 == 0 (checked on the host)
                const float4 cv = *reinterpret_cast<const float4 *>(c + d0);
                const float4 qv = *reinterpret_cast<const float4 *>(sq + d0);
                float t;
                t = qv.x - cv.x; dist[0] = dist[0] + t * t;
                t = qv.y - cv.y; dist[0] = dist[0] + t * t;
                t = qv.z - cv.z; dist[0] = dist[0] + t * t;
                t = qv.w - cv.w; dist[0] = dist[0] + t * t;
            }
        } else {
            // QN sums per row: the row in steps of 16 dimensions through two register buffers, the next step's 4
            // loads in flight while this step is summed (a row is one lane's; one load at a time waited out a memory
            // latency per 16 bytes)
            constexpr int SD = 16;
            float4 ba[SD / 4], bb[SD / 4];
            // unconditional loads (past the row end: its last 16 bytes again, never summed), so that the wait before a
            // step's sums counts only that step's loads
            auto load_step = [&](float4 (&v)[SD / 4], int d0) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < SD / 4; u++) v[u] = *reinterpret_cast<const float4 *>(c + min(d0 + 4 * u, d - 4));
            };
            auto sum_step = [&](const float4 (&v)[SD / 4], int d0) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < SD / 4; u++) {
                    if (d0 + 4 * u >= d) break;
#pragma unroll
                    for (int q = 0; q < QN; q++) {
                        const float4 qv = *reinterpret_cast<const float4 *>(sq + q * SCAN_D_MAX + d0 + 4 * u);
                        dist[q] = sq_acc(dist[q], qv.x, v[u].x);
                        dist[q] = sq_acc(dist[q], qv.y, v[u].y);
                        dist[q] = sq_acc(dist[q], qv.z, v[u].z);
                        dist[q] = sq_acc(dist[q], qv.w, v[u].w);
                    }
                }
            };
            load_step(ba, 0);
            for (int d0 = 0; d0 < d; d0 += 2 * SD) {
                load_step(bb, d0 + SD);
                sum_step(ba, d0);
                load_step(ba, d0 + 2 * SD);
                sum_step(bb, d0 + SD);
            }
        }
#pragma unroll
        for (int q = 0; q < QN; q++) {
            if (q >= nq) break;
            const float *qr = sq + q * SCAN_D_MAX;
            if (!kd_less(a.ko, qr, dist[q], (int)j, bd[q][K - 1], bi[q][K - 1])) continue;
            kd_list_insert<K>(a.ko, qr, bd[q], bi[q], dist[q], (int)j);  // keeps (distance, tie order)
        }
    }
    // per query: the workgroup's K best, K rounds of (distance, tie order) argmin over the threads' sorted lists
    for (int q = 0; q < nq; q++) {
        const float *qr = sq + q * SCAN_D_MAX;
        int ptr = 0;
        for (int r = 0; r < K; r++) {
            float v = INFINITY;
            int vi = 0x7fffffff;
#pragma unroll
            for (int x = 0; x < K; x++)
                if (x == ptr) {
                    v = bd[q][x];
                    vi = bi[q][x];
                }
            float mv = v;
            int mi = vi;
            kd_argmin<64>(a.ko, qr, mv, mi);
            if (lane == 0) {
                rd[w][r] = mv;
                ri[w][r] = mi;
            }
            if (vi == mi && mi != 0x7fffffff) ptr++;  // this wave's winner leaves its list
        }
        __syncthreads();
        if (w == 0) {  // merge the 4 waves' sorted K-lists: lane l < 4 holds wave l's list head
            int hp = 0;
            for (int r = 0; r < K; r++) {
                float v = INFINITY;
                int vi = 0x7fffffff;
                if (lane < 4 && hp < K) {
                    v = rd[lane][hp];
                    vi = ri[lane][hp];
                }
                float mv = v;
                int mi = vi;
                kd_argmin<64>(a.ko, qr, mv, mi);
                if (lane < 4 && vi == mi && mi != 0x7fffffff) hp++;
                if (lane == 0) {
                    const long o = ((long)(qg + q) * nsplit + blockIdx.x) * K + r;
                    pd[o] = mv;
                    pi[o] = mi;
                }
            }
        }
        __syncthreads();
    }
}

// The same scan on a mirror-orbit index (orbit.hip: every group holds a base row and up to 3 members that are exact
// signed permutations of it, (S_m c)[i] = +-c[src_m(i)] inside each 64-value colour component, the same map in all
// three): one wave takes 64 groups per round, one lane per group, and holds its group's base row in registers (from
// OrbitIndex::d_base, the fp32 base rows interleaved per 64-group block so every load is 1 KB contiguous).  The mirror
// tables are compile-time (orbitgen::MSRC / MNEG, checked against build_map when the index is built), so each member's
// value at dimension i is a fixed register, its sign a fixed add-or-subtract ((q - (-b)) == (q + b) bit for bit) and
// the query value a scalar operand: 3 VALU per (member, dimension).  Each member's sum runs in dimension order --
// the reference's sequential distance of its own row (orbit_eq_kernel checked row == S_m base with float equality; a
// -0 / +0 difference squares to the same term) -- so the lists are the row walk's bit for bit.
// ANN's order of two different present slots x, y of one group for query q (orbit.hip group_before)
__device__ __forceinline__ bool group_order_before(const GroupOrder *__restrict__ go, const float *__restrict__ q, int x,
                                                   int y) {
    const int lo = min(x, y), hi = max(x, y);
    const int pi = lo == 0 ? hi - 1 : lo == 1 ? hi + 1 : 5;  // (0,1)(0,2)(0,3)(1,2)(1,3)(2,3)
    const unsigned code = (go->pairs >> (3 * pi)) & 7u;
    const int node = code & 3;
    const bool lo_first = (q[go->cd[node]] - go->cv[node]) < 0.0f;
    const bool low_slot_first = ((code >> 2) & 1) == (unsigned)lo_first;
    return (x == lo) == low_slot_first;
}

template <int K>
__global__ __launch_bounds__(64) void nn_scan_orbit_kernel(RescoreArgs a, const float *__restrict__ qs,
                                                           const int4 *__restrict__ member,
                                                           const GroupOrder *__restrict__ gorder,
                                                           const float4 *__restrict__ base, long G, int nsplit,
                                                           float *__restrict__ pd, int *__restrict__ pi) {
    constexpr int D = 192;
    // workgroup = (64-group block, query), nsplit = the block count.  XCD-aware order: workgroups are dispatched
    // round-robin over the 8 XCDs (id % 8), so the nq workgroups of block b take ids on b's XCD, consecutively --
    // the block's rows are read from HBM once and from that XCD's L2 by the other queries
    const int lane = threadIdx.x, id = blockIdx.x, xcd = id & 7, slot = id >> 3, q = slot % a.nq;
    const long b = (long)(slot / a.nq) * 8 + xcd, g = b * 64 + lane;
    if (b >= nsplit) return;  // the padding of the block count to a multiple of 8
    const float *qr = qs + (long)q * D;  // uniform, restrict: the query values are scalar operands
    const int4 mj = g < G ? member[g] : make_int4(-1, -1, -1, -1);
    float cur[64];
    auto load = [&](int c, float *r) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const float4 v = base[(b * 48 + c * 16 + k) * 64 + lane];
            r[4 * k] = v.x;
            r[4 * k + 1] = v.y;
            r[4 * k + 2] = v.z;
            r[4 * k + 3] = v.w;
        }
    };
    load(0, cur);
    float dist[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    // components in a (not unrolled) loop: its 64 query values per component in scalar registers, the next
    // component's row values loading while this one is summed
    for (int c = 0; c < 3; c++) {
        float nxt[64];
        if (c < 2) load(c + 1, nxt);
        const float *qc = qr + c * 64;
#pragma unroll
        for (int i = 0; i < 64; i++) {
            const float qv = qc[i];
            const float t0 = qv - cur[i];
            dist[0] = dist[0] + t0 * t0;
#pragma unroll
            for (int m = 0; m < 3; m++) {
                const float bv = cur[orbitgen::MSRC[m][i]];
                const float t = orbitgen::MNEG[m][i] ? qv + bv : qv - bv;
                dist[m + 1] = dist[m + 1] + t * t;
            }
        }
        if (c < 2)
#pragma unroll
            for (int i = 0; i < 64; i++) cur[i] = nxt[i];
    }
    // the lane's (up to 4) members sorted by (distance, tie order) with a 4-input network (absent slots: the
    // (inf, 0x7fffffff) sentinel, which kd_less puts after every candidate), then K rounds of argmin over the wave
    // An exact tie between two members of the group is decided by the group's cached separating node
    // (GroupOrder, orbit.hip group_before: one compare) instead of kd_before's root-to-leaf walk.
    float bd[4] = {dist[0], dist[1], dist[2], dist[3]};
    int bi[4] = {mj.x, mj.y, mj.z, mj.w};
    int sl[4] = {0, 1, 2, 3};  // member slots, carried through the swaps
#pragma unroll
    for (int x = 0; x < 4; x++)
        if (bi[x] < 0) {
            bd[x] = INFINITY;
            bi[x] = 0x7fffffff;
        }
    const GroupOrder *go = gorder && g < G ? gorder + g : nullptr;
    auto cx = [&](int u, int w) {
        bool less;
        if (bd[w] != bd[u] || bi[w] == 0x7fffffff || bi[u] == 0x7fffffff || !go)
            less = kd_less(a.ko, qr, bd[w], bi[w], bd[u], bi[u]);
        else
            less = group_order_before(go, qr, sl[w], sl[u]);
        if (less) {
            const float td = bd[u];
            const int ti = bi[u], ts = sl[u];
            bd[u] = bd[w];
            bi[u] = bi[w];
            sl[u] = sl[w];
            bd[w] = td;
            bi[w] = ti;
            sl[w] = ts;
        }
    };
    cx(0, 1);
    cx(2, 3);
    cx(0, 2);
    cx(1, 3);
    cx(1, 2);
    int ptr = 0;
    for (int r = 0; r < K; r++) {
        float v = INFINITY;
        int vi = 0x7fffffff;
#pragma unroll
        for (int y = 0; y < 4; y++)
            if (y == ptr) {
                v = bd[y];
                vi = bi[y];
            }
        float mv = v;
        int mi = vi;
        kd_argmin<64>(a.ko, qr, mv, mi);
        if (vi == mi && mi != 0x7fffffff) ptr++;  // this lane's winner leaves its list
        if (lane == 0) {
            const long o = ((long)q * nsplit + b) * K + r;
            pd[o] = mv;
            pi[o] = mi;
        }
    }
}

// The k = 1 scan of a plain index, one wave per (candidate split, query): lane = row, the rows from the index's
// row-interleaved copy (NNIndex::d_rowsT, float4 piece k of row b * 64 + l at [b][k][l]: each load instruction reads
// 1 KB contiguous), the query values scalar operands (restrict pointer: scalar loads), 64 dimensions per step (d is a
// multiple of 64), the reference's sequential sum per row; each lane keeps its best (distance, tie order) over its rows, the wave's best
// goes to the merge.  XCD-aware order as nn_scan_orbit_kernel's (a split's queries on its XCD, consecutively).
__global__ __launch_bounds__(64) void nn_scan_rows_kernel(RescoreArgs a, const float *__restrict__ qs,
                                                          const float4 *__restrict__ rowsT, int nsplit,
                                                          float *__restrict__ pd, int *__restrict__ pi) {
    const int lane = threadIdx.x, id = blockIdx.x, xcd = id & 7, slot = id >> 3, q = slot % a.nq;
    const long sp = (long)(slot / a.nq) * 8 + xcd;
    if (sp >= nsplit) return;  // the padding of the split count to a multiple of 8
    const int d4 = a.d >> 2, nch = a.d >> 6;  // a.d % 64 == 0
    const long nb = ((long)a.n + 63) / 64;
    const long b0 = nb * sp / nsplit, b1 = nb * (sp + 1) / nsplit;
    const float *qr = qs + (long)q * a.d;
    float best = INFINITY;
    int bi = 0x7fffffff;
    for (long b = b0; b < b1; b++) {
        const float4 *rb = rowsT + b * d4 * 64 + lane;
        float dist = 0.0f;
        float4 cur[16];
        auto load = [&](int c, float4 *r) {
#pragma unroll
            for (int u = 0; u < 16; u++) r[u] = rb[(long)(c * 16 + u) * 64];
        };
        load(0, cur);
        // 64-dimension chunks in a (not unrolled) loop: the chunk's 64 query values in scalar registers, the next
        // chunk's 16 loads in flight while this one is summed
        for (int c = 0; c < nch; c++) {
            float4 nxt[16];
            if (c + 1 < nch) load(c + 1, nxt);
            const float *qk = qr + 64 * c;
#pragma unroll
            for (int u = 0; u < 16; u++) {
                float t = qk[4 * u] - cur[u].x;
                dist = dist + t * t;
                t = qk[4 * u + 1] - cur[u].y;
                dist = dist + t * t;
                t = qk[4 * u + 2] - cur[u].z;
                dist = dist + t * t;
                t = qk[4 * u + 3] - cur[u].w;
                dist = dist + t * t;
            }
            if (c + 1 < nch)
#pragma unroll
                for (int u = 0; u < 16; u++) cur[u] = nxt[u];
        }
        const int j = (int)(b * 64 + lane);
        if (j < a.n && kd_less(a.ko, qr, dist, j, best, bi)) {
            best = dist;
            bi = j;
        }
    }
    float mv = best;
    int mi = bi;
    kd_argmin<64>(a.ko, qr, mv, mi);
    if (lane == 0) {
        pd[(long)q * nsplit + sp] = mv;
        pi[(long)q * nsplit + sp] = mi;
    }
}

// rowsT = the row-interleaved copy of rows[n][d] (d % 4 == 0), zero past n
__global__ __launch_bounds__(256) void rows_interleave_kernel(const float4 *__restrict__ rows, long n, int d4,
                                                             float4 *__restrict__ rowsT) {
    const long total = (n + 63) / 64 * 64 * d4;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const long blk = t / (64L * d4);
        const int k = (int)(t / 64 % d4), l = (int)(t % 64);
        const long r = blk * 64 + l;
        rowsT[t] = r < n ? rows[r * d4 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// one 1024-thread workgroup per query (nsplit <= 1024, checked on the host), one split per thread: the k best of the
// query's nsplit * K partials (each split's list sorted) come from k rounds of (distance, tie order) argmin over the
// splits' list heads, across lanes and waves only -- no per-lane list.  Wave 0 then runs the common tail (results,
// tilemap item, ANN's pruning check, in-place replay).  Until round 5 a one-wave form kept up to 16 splits per lane in
// a per-lane K-list; its shifting insertion was miscompiled on exact ties (kdorder_dev.hpp kd_list_insert, DESIGN §4
// "A k = 8 correctness fix") and it was removed.
template <int K>
__global__ __launch_bounds__(1024) void nn_scan_merge_kernel(RescoreArgs a, int nsplit, const float *__restrict__ pd,
                                                             const int *__restrict__ pi) {
    const int q = blockIdx.x, lane = threadIdx.x & 63;
    const float *qr = a.q + (long)q * a.d;
    __shared__ float wd[16], rdw[32];
    __shared__ int wi[16], riw[32];
    {
        const int tid = threadIdx.x, w = tid >> 6;
        float hd[K];
        int hx[K];
#pragma unroll
        for (int r = 0; r < K; r++) {
            hd[r] = tid < nsplit ? pd[((long)q * nsplit + tid) * K + r] : INFINITY;
            hx[r] = tid < nsplit ? pi[((long)q * nsplit + tid) * K + r] : 0x7fffffff;
        }
        int hp = 0;
        for (int r = 0; r < a.k; r++) {
            float v = INFINITY;
            int vi = 0x7fffffff;
#pragma unroll
            for (int x = 0; x < K; x++)
                if (x == hp) {
                    v = hd[x];
                    vi = hx[x];
                }
            float mv = v;
            int mi = vi;
            kd_argmin<64>(a.ko, qr, mv, mi);
            if (lane == 0) {
                wd[w] = mv;
                wi[w] = mi;
            }
            __syncthreads();
            if (w == 0) {
                float v2 = lane < 16 ? wd[lane] : INFINITY;
                int i2 = lane < 16 ? wi[lane] : 0x7fffffff;
                kd_argmin<64>(a.ko, qr, v2, i2);
                if (lane == 0) {
                    rdw[r] = v2;
                    riw[r] = i2;
                }
            }
            __syncthreads();
            if (riw[r] != 0x7fffffff && vi == riw[r]) hp++;  // the winner's split moves to its next entry
        }
        if (w != 0) return;
    }
    int my_c = -1, first = -1;  // lane r keeps result r (the argmin is wave-uniform)
    float my_d = FLT_MAX, Dk = FLT_MAX;
    for (int r = 0; r < a.k; r++) {
        const float mv = rdw[r];
        const int mi = riw[r];
        const bool ok = mi != 0x7fffffff;
        if (lane == r) {
            my_c = ok ? mi : -1;
            my_d = ok ? mv : FLT_MAX;
        }
        if (r == 0) first = ok ? mi : -1;
        Dk = ok ? mv : FLT_MAX;
        if (lane == 0) {
            a.out_idx[(long)q * a.k + r] = ok ? mi : -1;
            a.out_err[(long)q * a.k + r] = ok ? mv : FLT_MAX;
            if (a.h_idx) {
                a.h_idx[(long)q * a.k + r] = ok ? mi : -1;
                a.h_err[(long)q * a.k + r] = ok ? mv : FLT_MAX;
            }
            if (r == 0) write_map(a, q, ok ? mi : -1);
        }
    }
    // ANN's pruning along every result's path (kd_verify_kernel's test): vouched for, or replayed exactly here by
    // lane 0 (kd_replay_query), which then rewrites the query's results and tilemap item.  Saves the root-box, verify
    // and replay launches of a coalesced per-tile batch: the wave forms the root box distance from registers, then
    // each half-wave walks one result's path, one level per lane (two results per pass).
    if (a.prune) {
        const KdOrder o = *a.ko;
        if (first >= 0 && Dk < FLT_MAX) {  // uniform
            const float rb = kd_root_box_wave(o, qr, lane);
            bool vouch = true;
            for (int r0 = 0; r0 < a.k; r0 += 2) {
                const int r = r0 + (lane >> 5);
                const int c = __shfl(my_c, r & 63, 64);
                const float dr = __shfl(my_d, r & 63, 64);
                const bool valid = r < a.k && (unsigned)c < (unsigned)o.n;
                const float fb = kd_half_path_far_box(o, qr, valid ? o.pos[c] : 0, rb, lane);
                if (r < a.k) vouch = vouch && valid && (fb < Dk || (fb <= Dk && dr == Dk));
            }
            const bool all = __all(vouch);
            if ((!all || a.force_replay) && lane == 0) {
                int *oi = a.out_idx + (long)q * a.k;
                float *oe = a.out_err + (long)q * a.k;
                const int best = kd_replay_query<K>(o, a.rows, qr, a.k, oi, oe);
                write_map(a, q, best);
                if (a.h_idx)
                    for (int r = 0; r < a.k; r++) {
                        a.h_idx[(long)q * a.k + r] = oi[r];
                        a.h_err[(long)q * a.k + r] = oe[r];
                    }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int pick_S(int d) {
    const int s = (d + 15) / 16;
    if (s <= 4) return 4;
    if (s <= 8) return 8;
    if (s <= 12) return 12;
    if (s <= 16) return 16;
    return 0;  // exact kernel only
}

NNIndex *nn_index_create_dev(float *d_rows, int n, int d, int bs, int split, hipStream_t stream) {
    NNIndex *ix = new NNIndex();
    ix->n = n;
    ix->d = d;
    ix->d_rows = d_rows;
    ix->bs = std::max(1, bs);
    ix->split = split;
    if (split == KD_SPLIT_STD && n > 0) {  // the reference's tree (main.pas:3779,3961): ANN's tie order
        ix->kd = kd_tree_build(d_rows, n, d, ix->bs, stream);
        if (!ix->kd) {
            nn_index_destroy(ix);
            return nullptr;
        }
    }
    ix->S = pick_S(d);
    ix->nblk = (n + 31) / 32;
    ix->h_fb_count = pinned_slot();
    if (!ix->h_fb_count) {
        set_error("nn_index_create_dev: pinned host allocation failed");
        nn_index_destroy(ix);
        return nullptr;
    }
    ix->h_fb_count[0] = 1 << 30;  // first call: full tier-2 grid
    ix->h_fb_count[1] = 0;
    if (ix->S == 0 || n == 0) return ix;
    // scale: power of two so that max|v| * scale <= 16384
    unsigned int *d_m = nullptr;
    DsStat *d_ds = nullptr;
    TILER_HIP_CHECK_NULL(dmalloc((void **)&d_m, 2 * sizeof(unsigned int)));
    TILER_HIP_CHECK_NULL(dmalloc((void **)&d_ds, sizeof(DsStat)));
    TILER_HIP_CHECK_NULL(hipMemsetAsync(d_m, 0, 2 * sizeof(unsigned int), stream));
    TILER_HIP_CHECK_NULL(hipMemsetAsync(d_ds, 0, sizeof(DsStat), stream));
    const long total = (long)n * d;
    hipLaunchKernelGGL(maxabs_kernel, dim3((unsigned)std::min<long>(2048, (total + 255) / 256)), dim3(256), 0, stream,
                       d_rows, total, d_m);
    unsigned int mbits[2] = {0, 0};
    TILER_HIP_CHECK_NULL(hipMemcpyAsync(mbits, d_m, sizeof(mbits), hipMemcpyDeviceToHost, stream));
    TILER_HIP_CHECK_NULL(hipStreamSynchronize(stream));
    float mabs;
    memcpy(&mabs, &mbits[0], 4);
    const bool all_int = mbits[1] == 0 && mabs <= 2048.0f;
    float scale = 1.0f;
    if (mabs > 0.0f && !all_int) {
        int e;
        frexpf(16384.0f / mabs, &e);
        scale = ldexpf(1.0f, e - 1);
    }
    ix->scale = scale;
    ix->perm = all_int ? 0 : 1;
    TILER_HIP_CHECK_NULL(dmalloc(&ix->d_frag, (size_t)ix->nblk * ix->S * 64 * 16));
    TILER_HIP_CHECK_NULL(dmalloc((void **)&ix->d_nc, (size_t)ix->nblk * 32 * sizeof(float)));
    TILER_HIP_CHECK_NULL(dmalloc((void **)&ix->d_seed, (size_t)ix->nblk * 32 * sizeof(float)));
    PrepArgs pa{d_rows, n, d, ix->S, scale, (half8 *)ix->d_frag, ix->d_nc, ix->d_seed, nullptr, d_ds, ix->perm};
    hipLaunchKernelGGL(prep_rows_kernel, dim3((unsigned)std::min<long>(4096, (ix->nblk + 3) / 4)), dim3(256), 0,
                       stream, pa);
    TILER_HIP_CHECK_NULL(hipGetLastError());
    DsStat ds;
    TILER_HIP_CHECK_NULL(hipMemcpyAsync(&ds, d_ds, sizeof(ds), hipMemcpyDeviceToHost, stream));
    TILER_HIP_CHECK_NULL(hipStreamSynchronize(stream));
    dfree(d_m);
    dfree(d_ds);
    auto bits2d = [](unsigned long long b) {
        double v;
        memcpy(&v, &b, 8);
        return v;
    };
    ix->maxN = sqrt(bits2d(ds.max_n2_bits));
    ix->maxH = sqrt(bits2d(ds.max_h2_bits));
    ix->maxE = sqrt(bits2d(ds.max_e2_bits));
    const double maxabs = bits2d(ds.max_abs_bits);
    ix->max_abs = maxabs;
    ix->exact_int = (ds.not_int == 0) && scale == 1.0f && maxabs <= 2048.0;
    if (ds.bad) ix->S = 0;  // non-finite / out-of-range data: exhaustive path only
    if (ix->S > 0 && ix->perm && (d + 31) / 32 == 6) {
        ix->S16 = 6;
        ix->nblk16 = (int)((n + 15) / 16);
        TILER_HIP_CHECK_NULL(dmalloc(&ix->d_frag16, (size_t)ix->nblk16 * ix->S16 * 1024));
        TILER_HIP_CHECK_NULL(dmalloc((void **)&ix->d_seed16, (size_t)ix->nblk16 * 16 * sizeof(float)));
        Prep16Args p16{d_rows, n, d, ix->S16, scale, (half8 *)ix->d_frag16, ix->d_seed16, 1, d == 192 ? 1 : 0};
        hipLaunchKernelGGL(prep16_kernel, dim3((unsigned)std::min<long>(4096, (ix->nblk16 + 3) / 4)), dim3(256), 0,
                           stream, p16);
        TILER_HIP_CHECK_NULL(hipGetLastError());
        TILER_HIP_CHECK_NULL(hipStreamSynchronize(stream));
    }
    if (ix->S > 0 && orbit_build(ix, stream) < 0) return nullptr;
    return ix;
}

void nn_scratch_free(SearchScratch &s, bool synced) {
    if (!synced && (s.qfrag || s.key || s.qrows || s.ccnt || s.fperm || s.kd_count))
        (void)hipDeviceSynchronize();  // dfree files the blocks for reuse: nothing may still read them (hipFree's rule)
    dfree(s.qfrag);
    dfree(s.qfrag16);
    dfree(s.qstat);
    dfree(s.key);
    dfree(s.idx);
    dfree(s.fb_list);
    dfree(s.fb_count);
    dfree(s.qrows);
    dfree(s.thr);
    dfree(s.gate);
    dfree(s.ex_list);
    dfree(s.ccnt);
    dfree(s.cbuf);
    dfree(s.kd_list);
    dfree(s.kd_count);
    dfree(s.kd_rootbox);
    dfree(s.kd_done);
    dfree(s.t2best);
    dfree(s.fperm);
    dfree(s.fbcnt);
    dfree(s.fcnt);
    dfree(s.fflag);
    dfree(s.fidx);
    dfree(s.ferr);
    dfree(s.ftile);
    dfree(s.fpal);
    dfree(s.fhm);
    dfree(s.fvm);
    s = SearchScratch();
}

void nn_index_destroy(NNIndex *ix) {
    if (!ix) return;
    (void)hipDeviceSynchronize();  // once for the whole index (dfree: hipFree's rule made explicit)
    orbit_destroy(ix->orbit, true);
    kd_tree_destroy(ix->kd, true);
    dfree(ix->d_rows);
    dfree(ix->d_rowsT);
    dfree(ix->d_frag);
    dfree(ix->d_nc);
    dfree(ix->d_seed);
    dfree(ix->d_frag16);
    dfree(ix->d_seed16);
    dfree(ix->d_tr_tile);
    dfree(ix->d_tr_pal);
    dfree(ix->d_tr_attr);
    nn_scratch_free(ix->scratch, true);
    pinned_slot_free(ix->h_fb_count);
    if (ix->done_event) hipEventDestroy(ix->done_event);
    delete ix;
}

static constexpr int TIER2_MAX = 65536;  // generic tier 2: queries per collect chunk (every tier-2 query has a slot)
static constexpr int TIER2_CAP = 1024;   // generic tier 2: collected candidates per query (beyond: tier 3)

static int ensure_scratch(NNIndex *ix, long nq, long nkeys) {
    SearchScratch &s = ix->scratch;
    // the outgrown buffers go back to the block cache: earlier searches must be done.  A handle's first call has
    // nothing to file, and a device-wide wait there would also wait for other streams' work (the encoder's next
    // Prepare, running beside this FrameTiling)
    const bool q_held = s.qfrag || s.qfrag16 || s.qstat || s.fb_list || s.fb_count || s.thr || s.gate || s.ex_list ||
                        s.kd_list || s.kd_rootbox || s.kd_done || s.t2best;
    if (((size_t)nq > s.cap_q && q_held) || ((size_t)nkeys > s.cap_keys && (s.key || s.idx)))
        (void)hipDeviceSynchronize();
    if ((size_t)nq > s.cap_q) {
        dfree(s.qfrag);
        dfree(s.qfrag16);
        dfree(s.qstat);
        dfree(s.fb_list);
        dfree(s.fb_count);
        dfree(s.thr);
        dfree(s.gate);
        dfree(s.ex_list);
        dfree(s.kd_list);
        dfree(s.kd_rootbox);
        dfree(s.kd_done);
        dfree(s.t2best);
        s.qfrag = s.qfrag16 = nullptr;
        s.qstat = nullptr;
        s.fb_list = s.fb_count = s.ex_list = s.kd_list = nullptr;
        s.thr = s.kd_rootbox = nullptr;
        s.gate = nullptr;
        s.kd_done = nullptr;
        s.t2best = nullptr;
        s.cap_q = 0;
        const long nqblk = (nq + 31) / 32 + 2;
        TILER_HIP_CHECK(dmalloc(&s.qfrag, (size_t)nqblk * 16 * 64 * 16));
        TILER_HIP_CHECK(dmalloc(&s.qfrag16, (size_t)((nq + 15) / 16 + 2) * 8 * 64 * 16));
        TILER_HIP_CHECK(dmalloc((void **)&s.qstat, (size_t)nq * sizeof(QStat)));
        TILER_HIP_CHECK(dmalloc((void **)&s.fb_list, (size_t)nq * sizeof(int)));
        TILER_HIP_CHECK(dmalloc((void **)&s.fb_count, 16));
        TILER_HIP_CHECK(dmalloc((void **)&s.thr, (size_t)nq * sizeof(float)));
        TILER_HIP_CHECK(dmalloc((void **)&s.gate, (size_t)nq * sizeof(float2)));
        TILER_HIP_CHECK(dmalloc((void **)&s.ex_list, (size_t)nq * sizeof(int)));
        TILER_HIP_CHECK(dmalloc((void **)&s.kd_list, (size_t)nq * sizeof(int)));
        TILER_HIP_CHECK(dmalloc((void **)&s.kd_rootbox, (size_t)nq * sizeof(float)));
        TILER_HIP_CHECK(dmalloc((void **)&s.kd_done, (size_t)nq));
        TILER_HIP_CHECK(dmalloc((void **)&s.t2best, (size_t)nq * sizeof(unsigned long long)));
        s.cap_q = nq;
    }
    if (!s.kd_count) TILER_HIP_CHECK(dmalloc((void **)&s.kd_count, 16));
    if ((size_t)nkeys > s.cap_keys) {
        dfree(s.key);
        dfree(s.idx);
        s.key = nullptr;
        s.idx = nullptr;
        s.cap_keys = 0;
        TILER_HIP_CHECK(dmalloc((void **)&s.key, (size_t)nkeys * sizeof(float)));
        TILER_HIP_CHECK(dmalloc((void **)&s.idx, (size_t)nkeys * sizeof(int)));
        s.cap_keys = nkeys;
    }
    return 0;
}

// waves per workgroup of the 32x32x16 shortlist on 64-d rows (UseOne's k = 8 preselection, main.pas:3830): two query
// blocks of 32 per wave, so 64 * NW queries per workgroup
static constexpr int GEN_NW_S4 = 4;
static constexpr int GEN_QB_S4 = 1;  // query blocks per wave there: 16,384 items x 4 splits fill 2 waves per SIMD
#ifndef GEN_QB_S4_BIG
#define GEN_QB_S4_BIG 2  // ... and from 32,768 items (whole-tileset keyframes: ~64k) two, each A fragment feeding 2 MFMAs
                         // (r06qb, profiles/r06/qb_preselect_qb2_encoder_ab.txt: whole-tileset loop 9.51 -> 9.59 Mtiles/s)
#endif
static int gen_qb_s4(int nq) { return nq >= 32768 ? GEN_QB_S4_BIG : GEN_QB_S4; }

template <int S, int L, int CB, int NW, int QB = 2>
static void launch_shortlist(NNIndex *ix, int nq, int nsplit, int bps, hipStream_t stream) {
    const int nqblk = (nq + 31) / 32;
    const dim3 grid((nqblk + QB * NW - 1) / (QB * NW), nsplit);
    const size_t lds = 2 * (CB * S * 1024 + CB * 128);
    KTimer tm("nn_shortlist", stream);
    hipLaunchKernelGGL((nn_shortlist_kernel<S, L, CB, NW, QB>), grid, dim3(NW * 64), lds, stream, (const half8 *)ix->d_frag,
                       ix->d_nc, ix->nblk, (const half8 *)ix->scratch.qfrag, nq, bps, nsplit, ix->perm,
                       ix->scratch.key, ix->scratch.idx);
}

// D=192 generic shortlist variant (A/B switch TILER_SHORTLIST, datasets without mirror orbits; C3 keyframe,
// one box): "q16" (default): nn_shortlist16_kernel, 16x16x32 MFMA, L16 = 4 (51.6 ms); "q16l6": L16 = 6
// (53.4 ms, fewer tier-2 queries); "w8": nn_shortlist_kernel, 32x32x16, 8 waves x 2 query blocks (63.9 ms)


static int shortlist_variant() {
    return 16;  // the shipped library: q16 only
}

// 16x16x32 shortlist for D = 161..192 float datasets: TILER_SHORTLIST=q16 (L16 = 4) / q16l6 (L16 = 6);
// returns L16, or 0 for the 32x32x16 kernels
// QB = 4 query blocks per wave; 5 (252 VGPRs) measured the same at 388k candidates (r03h: 80.6-81.2 vs 80.9-81.1 ms)
static constexpr int SL16_NW = 8, SL16_QB = 4, SL16_CB = 8;
// shortlist16_body VAR of the shipped kernel: the per-query-block insertion gate (r04c/r04e: -2..-3 % shortlist time,
// same digests; the 3-buffer ring, VAR 2, measured no gain)
static constexpr int SL16_VAR = 1;
static std::atomic<int> g_gate16{1};  // tiler_debug_shortlist_gate: the k = 1 insertion gate (A/B timing hook)
static int shortlist16_L() {
    const int v = shortlist_variant();
    return v == 16 ? 4 : v == 166 ? 6 : 0;
}

template <int S, int L>
static int launch_shortlist16(NNIndex *ix, int nq, int nsplit, int bps, bool gated, hipStream_t stream) {
    const int nqblk = (nq + 15) / 16;
    const dim3 grid((nqblk + SL16_NW * SL16_QB - 1) / (SL16_NW * SL16_QB), nsplit);
    const size_t buf = SL16_CB * S * 1024 + SL16_CB * 64;
    float gb = 0.0f;
    if (gated) {  // the k = 1 gate (gate16_kernel): per query (x, y) from the query statistics, gb = (1 + g)/(1 - g)
        const double u = 5.9604644775390625e-08;
        const double g = (double)(ix->d + 4) * u / (1.0 - (double)(ix->d + 4) * u) * 1.05;
        const double b = (1.0 + g) / (1.0 - g);
        gb = (float)b;
        if ((double)gb < b) gb = nextafterf(gb, INFINITY);
        hipLaunchKernelGGL(gate16_kernel, dim3((nq + 255) / 256), dim3(256), 0, stream, ix->scratch.qstat, nq, ix->d,
                           ix->maxN, ix->maxH, ix->maxE, ix->scratch.gate);
    }
    auto go = [&](auto kern, int nbuf) {
        hipLaunchKernelGGL(kern, grid, dim3(SL16_NW * 64), nbuf * buf, stream, (const half8 *)ix->d_frag16,
                           ix->d_seed16, ix->nblk16, (const half8 *)ix->scratch.qfrag16, nq, bps, nsplit, ix->perm,
                           ix->scratch.key, ix->scratch.idx, ix->flat_cnt, gated ? (const float2 *)ix->scratch.gate : nullptr,
                           gb);
    };
    KTimer tm("nn_shortlist", stream);
    go(nn_shortlist16_kernel<S, L, SL16_CB, SL16_NW, SL16_QB, 0, SL16_VAR>, 2);
    TILER_HIP_CHECK(hipGetLastError());
    if (ix->flat_cnt) {  // flat_queries of the stats: derived from the device count when they are read
        ix->last_flat_dev = ix->flat_cnt;
        ix->last_flat_nq = nq;
        ix->last_flat_qpw = SL16_NW * SL16_QB * 16;
        ix->last_flat_wgs = grid.x;
    }
    return 0;
}

template <int L>
static int dispatch_shortlist(NNIndex *ix, int nq, int nsplit, int bps, hipStream_t stream) {
    switch (ix->S) {
        case 4:
            if (gen_qb_s4(nq) == 2)
                launch_shortlist<4, L, 6, GEN_NW_S4, 2>(ix, nq, nsplit, bps, stream);
            else
                launch_shortlist<4, L, 6, GEN_NW_S4, GEN_QB_S4>(ix, nq, nsplit, bps, stream);
            break;
        case 8: launch_shortlist<8, L, 3, 4>(ix, nq, nsplit, bps, stream); break;
        case 12: launch_shortlist<12, L, 2, 8>(ix, nq, nsplit, bps, stream); break;
        case 16: launch_shortlist<16, L, 2, 4>(ix, nq, nsplit, bps, stream); break;
        default: set_error("nn: unsupported fragment depth"); return -1;
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

template <int S, int CB>
static void launch_collect(NNIndex *ix, int nq, int jbase, hipStream_t stream) {
    // fixed grid (the overflow count stays on the device): many short splits so that a few hundred
    // overflowed queries still spread over the whole chip; grid.x strides over the chunk's query groups of 256,
    // so 2 x 256 resident-sized workgroups serve any count alike
    const int nsplit = std::min(ix->nblk, 256);
    const int bps = (ix->nblk + nsplit - 1) / nsplit;
    const int groups = std::min(2, (std::min(nq - jbase, TIER2_MAX) + 255) / 256);
    const size_t lds = 2 * (CB * S * 1024 + CB * 128);
    SearchScratch &s = ix->scratch;
    KTimer tm("nn_collect", stream);
    hipLaunchKernelGGL((nn_collect_kernel<S, CB>), dim3(groups, (ix->nblk + bps - 1) / bps), dim3(256), lds, stream,
                       (const half8 *)ix->d_frag, ix->d_nc, ix->nblk, (const half8 *)s.qfrag, s.fb_list, s.fb_count,
                       jbase, TIER2_MAX, s.thr, bps, ix->perm, s.ccnt, s.cbuf, TIER2_CAP);
}

static int dispatch_collect(NNIndex *ix, int nq, int jbase, hipStream_t stream) {
    switch (ix->S) {
        case 4: launch_collect<4, 6>(ix, nq, jbase, stream); break;
        case 8: launch_collect<8, 3>(ix, nq, jbase, stream); break;
        case 12: launch_collect<12, 2>(ix, nq, jbase, stream); break;
        case 16: launch_collect<16, 2>(ix, nq, jbase, stream); break;
        default: set_error("nn: unsupported fragment depth"); return -1;
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

static int launch_exact(RescoreArgs ra, int list_n, int grid, hipStream_t stream) {
    if (ra.d > 1024) {
        set_error("nn: dimension > 1024 unsupported");
        return -1;
    }
    KTimer tm("nn_exact", stream);
    if (ra.k <= 1)
        hipLaunchKernelGGL(nn_exact_kernel<1>, dim3(grid), dim3(256), 0, stream, ra, list_n);
    else if (ra.k <= 8)
        hipLaunchKernelGGL(nn_exact_kernel<8>, dim3(grid), dim3(256), 0, stream, ra, list_n);
    else if (ra.k <= 32)
        hipLaunchKernelGGL(nn_exact_kernel<32>, dim3(grid), dim3(256), 0, stream, ra, list_n);
    else {
        set_error("nn: k > 32 unsupported");
        return -1;
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

static int search_tail(NNIndex *ix, const RescoreArgs &ra, int nq, hipStream_t stream, const OrbitTail *orbit);

// generic tier-2 slots of a search: whole chunks covering 1.5x the largest tier-2 count of the recent searches (this
// index's last count, or the last one seen on any index: an encoder builds a new index per keyframe), >= 1 chunk.
// A fresh index (the 1 << 30 sentinel: no search of its own yet) takes 3x the recent count of the other indexes, a
// margin for an unrelated one.  Queries past the slots go to the exhaustive tier 3: exact either way, slower.
static std::atomic<int> g_t2_recent{0};
static int tier2_slots(NNIndex *ix, int nq) {
    const int own = ix->h_fb_count ? ((volatile int *)ix->h_fb_count)[0] : 0;
    const bool fresh = own >= (1 << 30);
    const int recent = g_t2_recent.load(std::memory_order_relaxed);
    const int prev = fresh ? 2 * recent : std::max(own, recent);
    const long want = (long)prev + prev / 2 + 1;
    const long chunks = std::max(1L, (want + TIER2_MAX - 1) / TIER2_MAX);
    return (int)std::min<long>(nq, chunks * TIER2_MAX);
}
static int search_core(NNIndex *ix, RescoreArgs &ra, const float *d_q, int nq, int k, hipStream_t stream,
                       bool orbit_prepared);
static bool scan_small_takes(const NNIndex *ix, int nq, int k);
static std::atomic<int> g_force_replay{0};  // tiler_debug_force_replay

int nn_search_dev(NNIndex *ix, const float *d_q, int nq, int k, int *d_idx, float *d_err, const FtMaps *maps,
                  hipStream_t stream, bool rootbox_ready, bool orbit_prepared, int *h_idx, float *h_err) {
    if (nq <= 0) return 0;
    if (k < 1 || k > 32) {
        set_error("nn: k must be in 1..32");
        return -1;
    }
    RescoreArgs ra{};
    ra.rows = ix->d_rows;
    ra.q = d_q;
    ra.n = ix->n;
    ra.d = ix->d;
    ra.nq = nq;
    ra.k = k;
    ra.N = ix->maxN;
    ra.H = ix->maxH;
    ra.Ec = ix->maxE;
    ra.ds_int = ix->exact_int ? 1 : 0;
    ra.max_abs_c = ix->max_abs;
    ra.out_idx = d_idx;
    ra.out_err = d_err;
    ra.ko = ix->kd ? ix->kd->d_view : nullptr;
    ra.h_idx = h_idx;
    ra.h_err = h_idx ? h_err : nullptr;
    if (maps && k == 1 && ix->d_tr_tile) {
        ra.tr_tile = ix->d_tr_tile;
        ra.tr_pal = ix->d_tr_pal;
        ra.tr_attr = ix->d_tr_attr;
        ra.m_tile = maps->tile;
        ra.m_pal = maps->pal;
        ra.m_hm = maps->hm;
        ra.m_vm = maps->vm;
    }
    ix->last_queries = nq;
    ix->last_flat_dev = nullptr;
    SearchScratch &s = ix->scratch;
    if (!ix->done_event) TILER_HIP_CHECK(hipEventCreateWithFlags(&ix->done_event, hipEventDisableTiming));
    if (ix->kd && scan_small_takes(ix, nq, k)) {  // the coalesced per-tile batches: scan, merge + pruning check, replay
        if (ensure_scratch(ix, nq, 0)) return -1;
        ra.prune = ix->kd->n > ix->kd->bs;  // a single bucket: no pruning, position order is exact
        ra.force_replay = g_force_replay.load(std::memory_order_relaxed);
        if (search_core(ix, ra, d_q, nq, k, stream, orbit_prepared)) return -1;
        TILER_HIP_CHECK(hipEventRecord(ix->done_event, stream));
        return 0;
    }
    if (ix->kd) {  // ANN's tie order: the pruning check needs every query's box distance and a clean slate
        if (ensure_scratch(ix, nq, 0)) return -1;
        if (!rootbox_ready) {  // the box distances, with the verify flags and the replay count cleared in the same launch
            if (kd_root_boxes(ix->kd, d_q, nq, s.kd_rootbox, stream, s.kd_done, s.kd_count)) return -1;
        } else {
            TILER_HIP_CHECK(hipMemsetAsync(s.kd_done, 0, (size_t)nq, stream));
            TILER_HIP_CHECK(hipMemsetAsync(s.kd_count, 0, sizeof(int), stream));
        }
    }
    if (search_core(ix, ra, d_q, nq, k, stream, orbit_prepared)) return -1;
    if (!ix->kd) {
        TILER_HIP_CHECK(hipEventRecord(ix->done_event, stream));
        return 0;
    }
    // ANN's box pruning along every result's path (queries the pair pass did not already check); the rare query
    // it cannot vouch for is replayed exactly
    KdFixArgs fa{ix->d_rows, d_q, nq, k, d_idx, d_err};
    fa.rootbox = s.kd_rootbox;
    fa.done = s.kd_done;
    fa.tr_tile = ra.tr_tile;
    fa.tr_pal = ra.tr_pal;
    fa.tr_attr = ra.tr_attr;
    fa.m_tile = ra.m_tile;
    fa.m_pal = ra.m_pal;
    fa.m_hm = ra.m_hm;
    fa.m_vm = ra.m_vm;
    fa.list = s.kd_list;
    fa.count = s.kd_count;
    fa.force_replay = g_force_replay.load(std::memory_order_relaxed);
    if (kd_verify_and_replay(ix->kd, fa, stream)) return -1;
    TILER_HIP_CHECK(hipEventRecord(ix->done_event, stream));  // what tiler_search_stats reads is final here
    return 0;
}

// the small-batch path (nn_scan_small_kernel): groups of up to 16 queries (k = 1) or 4 (k <= 8) per workgroup row,
// batches of up to SCAN_MAX1 / SCAN_MAX8 queries
static constexpr int SCAN_QN1 = 16, SCAN_QN8 = 4;
static constexpr long SCAN_ROWS_MAXN = 65536;   // nn_scan_rows_kernel up to this many candidates
static constexpr long SCAN_ORB_MAXBLK = 1024;  // the orbit scan's splits (64-group blocks) at most: the wide merge's
static std::atomic<int> g_scan_max1{64}, g_scan_max8{16};  // tiler_set_scan_limits
void nn_set_scan_limits(int max_k1, int max_k8) {
    g_scan_max1.store(std::max(0, max_k1));
    g_scan_max8.store(std::max(0, max_k8));
}
void nn_set_force_replay(int on) { g_force_replay.store(on != 0); }
void nn_set_shortlist_gate(int on) { g_gate16.store(on != 0); }
bool nn_search_is_small(const NNIndex *ix, int nq, int k) { return scan_small_takes(ix, nq, k); }
static bool scan_small_takes(const NNIndex *ix, int nq, int k) {
    return ix->d <= SCAN_D_MAX && ix->d % 4 == 0 &&
           ((k == 1 && nq <= g_scan_max1.load(std::memory_order_relaxed)) ||
            (k <= 8 && nq <= g_scan_max8.load(std::memory_order_relaxed)));
}
static int scan_small(NNIndex *ix, RescoreArgs &ra, int nq, int k, hipStream_t stream) {
    const OrbitIndex *o = ix->orbit;
    // mirror orbits: base rows only (nn_scan_orbit_kernel), one wave per (64-group block, query)
    const long nblk = o ? ((long)o->G + 63) / 64 : 0;
    const bool orb = o && o->d_base && o->G > 0 && ix->d == 192 && nblk <= SCAN_ORB_MAXBLK;
    const int K = k == 1 ? 1 : 8;
    // k = 1 on a plain index: the row-interleaved scan (nn_scan_rows_kernel); its copy is made on first use and waited
    // for (a concurrent slot's scan may be queued on another stream as soon as this call releases the index)
    // (at larger n the split-per-thread scan reads each row once for the batch's queries at near HBM peak: r05w2, the
    // shuffled 262,144-row handle, 1 query 73 vs 77 us, batches slower)
    const bool rows_scan = !orb && K == 1 && ix->d % 64 == 0 && ix->n <= SCAN_ROWS_MAXN;
    if (rows_scan && !ix->d_rowsT) {
        const long nb = ((long)ix->n + 63) / 64;
        TILER_HIP_CHECK(dmalloc((void **)&ix->d_rowsT, (size_t)nb * 64 * ix->d * sizeof(float)));
        hipLaunchKernelGGL(rows_interleave_kernel, dim3((unsigned)std::min<long>(8192, (nb * 64 * (ix->d / 4) + 255) / 256)),
                           dim3(256), 0, stream, (const float4 *)ix->d_rows, (long)ix->n, ix->d / 4, (float4 *)ix->d_rowsT);
        TILER_HIP_CHECK(hipGetLastError());
        TILER_HIP_CHECK(hipStreamSynchronize(stream));
    }
    const int nsplit = orb ? (int)nblk
                           : rows_scan ? (int)std::max<long>(1, ((long)ix->n + 63) / 64)
                                       : (int)std::max<long>(1, std::min<long>(1024, ((long)ix->n + 255) / 256));
    if (nsplit > 1024) {  // the merge holds one split per thread of one workgroup (the caps above keep this)
        set_error("scan_small: " + std::to_string(nsplit) + " candidate splits exceed the merge's 1024");
        return -1;
    }
    if (ensure_scratch(ix, nq, (long)nq * nsplit * K)) return -1;
    SearchScratch &s = ix->scratch;
    ix->last_splits = 0;  // the stats report no tier-2 / tier-3 queries for a scan (fb_count is not read)
    ix->last_fallback = 0;
    KTimer tm("nn_scan", stream);
    // the per-query work is unrolled over QN: the smallest instance that holds a group
    const int qn = K == 1 ? (nq == 1 ? 1 : nq <= 4 ? 4 : SCAN_QN1) : (nq == 1 ? 1 : SCAN_QN8);
    const dim3 grid(nsplit, (nq + qn - 1) / qn);
    auto scan = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, ra, nsplit, s.key, s.idx);
    };
    auto scan_o = [&](auto kern) {  // one wave per (64-group block, query), the block count padded to 8 XCDs
        hipLaunchKernelGGL(kern, dim3((unsigned)(((nsplit + 7) / 8) * 8 * nq)), dim3(64), 0, stream, ra, ra.q,
                           (const int4 *)o->d_member, ra.ko && ix->kd && ix->kd->bs == 1 ? (const GroupOrder *)o->d_gorder : nullptr,
                           (const float4 *)o->d_base, (long)o->G, nsplit, s.key, s.idx);
    };
    // the merge: one split per thread (cross-lane selection only)
    auto merge = [&]() {
        const float *pk = s.key;
        const int *pj = s.idx;
        if (K == 1)
            hipLaunchKernelGGL(nn_scan_merge_kernel<1>, dim3(nq), dim3(1024), 0, stream, ra, nsplit, pk, pj);
        else
            hipLaunchKernelGGL(nn_scan_merge_kernel<8>, dim3(nq), dim3(1024), 0, stream, ra, nsplit, pk, pj);
    };
    if (orb) {
        if (K == 1) scan_o(nn_scan_orbit_kernel<1>);
        else scan_o(nn_scan_orbit_kernel<8>);
    } else if (rows_scan) {
        hipLaunchKernelGGL(nn_scan_rows_kernel, dim3((unsigned)(((nsplit + 7) / 8) * 8 * nq)), dim3(64), 0, stream, ra,
                           ra.q, (const float4 *)ix->d_rowsT, nsplit, s.key, s.idx);
    } else if (K == 1) {
        if (qn == 1) scan(nn_scan_small_kernel<1, 1>);
        else if (qn == 4) scan(nn_scan_small_kernel<4, 1>);
        else scan(nn_scan_small_kernel<SCAN_QN1, 1>);
    } else {
        if (qn == 1) scan(nn_scan_small_kernel<1, 8>);
        else scan(nn_scan_small_kernel<SCAN_QN8, 8>);
    }
    merge();
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

static int search_core(NNIndex *ix, RescoreArgs &ra, const float *d_q, int nq, int k, hipStream_t stream,
                       bool orbit_prepared) {
    if (scan_small_takes(ix, nq, k)) return scan_small(ix, ra, nq, k, stream);
    const bool mfma = ix->S > 0 && k <= 8;
    if (!mfma) {
        ix->last_splits = 0;
        ix->last_fallback = nq;
        ra.ex_list = nullptr;
        return launch_exact(ra, nq, std::min(nq, 4096), stream);
    }
    // 32x32x16 shortlist: 2 lanes x L = 8 per query (>= 2x the 4-way mirror near-ties of one tile per
    // lane, row_perm spreads them 2+2); 16x16x32: 4 lanes x L16 (perm16 spreads them 1 per lane)
    const int v16 = ix->S16 > 0 ? shortlist16_L() : 0;
    const int L = v16 ? v16 : 8;
    const int lpq = v16 ? 4 : 2;
    const int nblk = v16 ? ix->nblk16 : ix->nblk;
    const int max_split = 64 / (lpq * L);
    const int qpwg = v16 ? SL16_NW * SL16_QB * 16 : (ix->S == 12 ? 512 : ix->S == 4 ? 32 * gen_qb_s4(nq) * GEN_NW_S4 : 256);
    const int wgs = (nq + qpwg - 1) / qpwg;
    int nsplit = std::max(1, std::min(max_split, (1024 + wgs - 1) / wgs));
    nsplit = std::min(nsplit, nblk);
    const int bps = (nblk + nsplit - 1) / nsplit;
    nsplit = (nblk + bps - 1) / bps;
    ix->last_splits = nsplit;
    if (ensure_scratch(ix, nq, (long)nq * nsplit * lpq * L)) return -1;
    SearchScratch &s = ix->scratch;
    TILER_HIP_CHECK(hipMemsetAsync(s.fb_count, 0, 16, stream));
    ix->last_orbit = 0;
    if (k == 1 && ix->orbit) {
        // mirror-orbit path (orbit.hip): tier 2 lists every query the rescore cannot settle (fb_max = nq)
        OrbitTail t{};
        t.fb_list = s.fb_list;
        t.fb_count = s.fb_count;
        t.ex_list = s.ex_list;
        t.ex_count = s.fb_count + 1;
        t.fb_max = nq;
        t.thr = s.thr;
        t.t2_best = s.t2best;
        t.flat_cnt = ix->flat_cnt;
        t.out_idx = ra.out_idx;
        t.out_err = ra.out_err;
        t.tr_tile = ra.tr_tile;
        t.tr_pal = ra.tr_pal;
        t.tr_attr = ra.tr_attr;
        t.m_tile = ra.m_tile;
        t.m_pal = ra.m_pal;
        t.m_hm = ra.m_hm;
        t.m_vm = ra.m_vm;
        t.ko = ra.ko;
        t.kd_rootbox = s.kd_rootbox;
        t.kd_done = s.kd_done;
        t.kd_list = s.kd_list;
        t.kd_count = s.kd_count;
        if (orbit_search(ix, d_q, nq, t, stream, orbit_prepared && k == 1)) return -1;
        ix->last_orbit = 1;
        ra.qstat = s.qstat;
        ra.fb_list = s.fb_list;
        ra.fb_count = s.fb_count;
        ra.ex_list = s.ex_list;
        ra.ex_count = s.fb_count + 1;
        ra.thr = s.thr;
        ra.fb_max = nq;
        return search_tail(ix, ra, nq, stream, &t);
    }
    // queries -> fragments (same layout and scale as the dataset)
    const long nqblk = (nq + 31) / 32;
    PrepArgs pa{d_q, nq, ix->d, ix->S, ix->scale, (half8 *)s.qfrag, nullptr, nullptr, s.qstat, nullptr, 0};
    {
        KTimer t_prep("nn_prep", stream);
        hipLaunchKernelGGL(prep_rows_kernel, dim3((unsigned)std::min<long>(4096, (nqblk + 3) / 4)), dim3(256), 0,
                           stream, pa);
    }
    TILER_HIP_CHECK(hipGetLastError());
    if (v16) {
        Prep16Args p16{d_q, nq, ix->d, ix->S16, ix->scale, (half8 *)s.qfrag16, nullptr, 0, ix->d == 192 ? 1 : 0};
        {
            KTimer t_prep("nn_prep", stream);
            hipLaunchKernelGGL(prep16_kernel, dim3((unsigned)std::min<long>(4096, ((nq + 15) / 16 + 3) / 4)),
                               dim3(256), 0, stream, p16);
        }
        TILER_HIP_CHECK(hipGetLastError());
        {
            if (launch_shortlist16<6, 4>(ix, nq, nsplit, bps, k == 1 && g_gate16.load(std::memory_order_relaxed), stream))
                return -1;
        }
    } else if (dispatch_shortlist<8>(ix, nq, nsplit, bps, stream)) {
        return -1;
    }
    ra.qstat = s.qstat;
    ra.key = s.key;
    ra.idx = s.idx;
    ra.L = L;
    ra.lpq = lpq;
    ra.nsplit = nsplit;
    ra.fb_list = s.fb_list;
    ra.fb_count = s.fb_count;
    ra.ex_list = s.ex_list;
    ra.ex_count = s.fb_count + 1;
    ra.thr = s.thr;
    if (!s.ccnt) {  // the generic tier 2's collect buffers (256 MB), on the first search that can need them
        TILER_HIP_CHECK(dmalloc((void **)&s.ccnt, (size_t)TIER2_MAX * sizeof(int)));
        TILER_HIP_CHECK(dmalloc((void **)&s.cbuf, (size_t)TIER2_MAX * TIER2_CAP * sizeof(int)));
    }
    ra.ccnt = s.ccnt;
    ra.cbuf = s.cbuf;
    ra.cap = TIER2_CAP;
    // tier-2 slots: the collect runs in chunks of TIER2_MAX, as many as the recent tier-2 counts call for (each
    // chunk costs two launches even when empty); an overflowed query beyond the slots goes to the exact tier 3, so
    // the count only shapes the work, never the result
    ra.fb_max = tier2_slots(ix, nq);
    TILER_HIP_CHECK(hipMemsetAsync(s.ccnt, 0, (size_t)std::min(nq, TIER2_MAX) * sizeof(int), stream));
    {
        KTimer t_rs("nn_rescore", stream);
        if (ra.nsplit * ra.lpq * ra.L <= 16)
            hipLaunchKernelGGL(nn_rescore_kernel<16>, dim3((nq + 15) / 16), dim3(256), 0, stream, ra);
        else
            hipLaunchKernelGGL(nn_rescore_kernel<64>, dim3((nq + 3) / 4), dim3(256), 0, stream, ra);
    }
    TILER_HIP_CHECK(hipGetLastError());
    return search_tail(ix, ra, nq, stream, nullptr);
}

// tiers 2 and 3 read their device-side counts: fixed grids, no host round trip.  Every query the rescore cannot
// settle has a tier-2 slot whatever their number: the orbit tier 2 has no per-query buffer to overflow, the generic
// one runs its slots in chunks of TIER2_MAX (a chunk past the device count exits at once).  Tier 3, the exhaustive
// scan, is left to non-finite / fp16-overflowing queries (and generic buffer overflows); its grid fills the chip.
static int search_tail(NNIndex *ix, const RescoreArgs &ra, int nq, hipStream_t stream, const OrbitTail *orbit) {
    SearchScratch &s = ix->scratch;
    if (orbit) {
        if (orbit_tier2(ix, ra.q, *orbit, nq, stream)) return -1;
    } else {
        for (int jbase = 0; jbase < ra.fb_max; jbase += TIER2_MAX) {
            if (dispatch_collect(ix, nq, jbase, stream)) return -1;
            KTimer t_r2("nn_rescore2", stream);
            hipLaunchKernelGGL(nn_rescore2_kernel,
                               dim3((unsigned)std::min(1024, (std::min(nq - jbase, TIER2_MAX) + 3) / 4)), dim3(256), 0,
                               stream, ra, jbase, TIER2_MAX);
            TILER_HIP_CHECK(hipGetLastError());
        }
    }
    if (launch_exact(ra, 0, std::min(nq, 1024), stream)) return -1;
    TILER_HIP_CHECK(hipMemcpyAsync(ix->h_fb_count, s.fb_count, 2 * sizeof(int), hipMemcpyDeviceToHost, stream));
    if (!orbit) {  // a heuristic only: the copy above is still in flight, so this reads the previous search's count
        // on this index (or, racing the DMA, this one's; the sentinel on a fresh index is skipped)
        const int c = ((volatile int *)ix->h_fb_count)[0];
        if (c >= 0 && c < (1 << 30)) g_t2_recent.store(c, std::memory_order_relaxed);
    }
    return 0;
}

// Flat tiles (one colour: every Haar coefficient but the DC is 0, so only isotypic block 0 of q' is nonzero) are
// moved to the end of the batch, where whole shortlist workgroups of them run 3 of the 12 k-steps (orbit_search).
// A: per tile flag + per-block count of the others; B: one workgroup scans the block counts; C: stable positions
// (others first, flats after, each in tile order), which the query kernel reads through; D: the outputs back.
__global__ __launch_bounds__(256) void ft_flat_flag_kernel(const int32_t *__restrict__ rgb, int Q, uint8_t *flag,
                                                           int *bcnt) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    int other = 0;
    if (i < Q) {
        const int4 *t = reinterpret_cast<const int4 *>(rgb + i * 64);
        const int c0 = rgb[i * 64];
        bool flat = true;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int4 v = t[k];
            flat = flat && v.x == c0 && v.y == c0 && v.z == c0 && v.w == c0;
        }
        flag[i] = flat ? 1 : 0;
        other = flat ? 0 : 1;
    }
    const int c = __syncthreads_count(other);
    if (threadIdx.x == 0) bcnt[blockIdx.x] = c;
}

__global__ __launch_bounds__(1024) void ft_flat_scan_kernel(int *bcnt, int nb, int *total) {
    __shared__ int sc[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int b0 = 0; b0 < nb; b0 += 1024) {
        const int b = b0 + threadIdx.x;
        const int v = b < nb ? bcnt[b] : 0;
        sc[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int u = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
            __syncthreads();
            sc[threadIdx.x] += u;
            __syncthreads();
        }
        if (b < nb) bcnt[b] = carry + sc[threadIdx.x] - v;  // exclusive prefix
        __syncthreads();
        if (threadIdx.x == 1023) carry += sc[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void ft_flat_place_kernel(const int32_t *__restrict__ rgb, int Q,
                                                            const uint8_t *__restrict__ flag,
                                                            const int *__restrict__ boff, const int *__restrict__ total,
                                                            int *perm) {
    __shared__ int sc[256];
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const int f = i < Q ? flag[i] : 1;
    sc[threadIdx.x] = f ? 0 : 1;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int u = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
        __syncthreads();
        sc[threadIdx.x] += u;
        __syncthreads();
    }
    if (i >= Q) return;
    const int rank_other = sc[threadIdx.x] - (f ? 0 : 1);          // others before this tile in the block
    const int rank_flat = (int)threadIdx.x - rank_other - (f ? 0 : 1);  // flats before it in the block
    const int b_other = boff[blockIdx.x], b_flat = (int)(blockIdx.x * 256) - b_other;
    const long pos = f ? (long)*total + b_flat + rank_flat : (long)b_other + rank_other;
    perm[pos] = (int)i;  // the query kernel reads tile perm[pos] (no copy of the RGB)
}

__global__ __launch_bounds__(256) void ft_unpermute_kernel(int Q, const int *__restrict__ perm, const int *fidx,
                                                           const float *ferr, const int32_t *ftile, const int32_t *fpal,
                                                           const uint8_t *fhm, const uint8_t *fvm, int *idx, float *err,
                                                           FtMaps maps) {
    const long p = (long)blockIdx.x * 256 + threadIdx.x;
    if (p >= Q) return;
    const long o = perm[p];
    if (idx) idx[o] = fidx[p];
    if (err) err[o] = ferr[p];
    if (maps.tile) maps.tile[o] = ftile[p];
    if (maps.pal) maps.pal[o] = fpal[p];
    if (maps.hm) maps.hm[o] = fhm[p];
    if (maps.vm) maps.vm[o] = fvm[p];
}

int nn_frame_tiling_dev(NNIndex *ix, const int32_t *d_rgb, int Q, int use_wavelets, int gamma, int *d_idx,
                        float *d_err, const FtMaps *maps, hipStream_t stream) {
    if (Q <= 0) return 0;
    if (ix->d != 192) {
        set_error("frame tiling: dataset dimension must be 192 (cTileDCTSize)");
        return -1;
    }
    SearchScratch &s = ix->scratch;
    if ((size_t)Q > s.cap_rows) {
        if (s.qrows) (void)hipDeviceSynchronize();  // the outgrown buffer goes back to the block cache (ensure_scratch)
        dfree(s.qrows);
        s.qrows = nullptr;
        s.cap_rows = 0;
        TILER_HIP_CHECK(dmalloc((void **)&s.qrows, (size_t)Q * 192 * sizeof(float)));
        s.cap_rows = Q;
    }
    const bool fuse_rb = ix->kd && use_wavelets && ix->kd->dd == 192;
    if (fuse_rb && ensure_scratch(ix, Q, 0)) return -1;
    constexpr bool noflat = false;
    // flat grouping on the generic path (datasets without mirror orbits: real PrepareFrameTiling candidate sets):
    // the 16x16x32 shortlist's flat workgroups contract k-step 0 only (dc_first_dim)
    const bool flat_generic = !ix->orbit && use_wavelets && ix->S16 > 0 && shortlist16_L() > 0 && Q >= 8192;
    if (flat_generic || (ix->orbit && use_wavelets)) {
        // flat tiles last (see ft_flat_flag_kernel) when the shortlist is long enough to repay the ~0.1 ms of
        // grouping: C3 (2,048 group blocks) -0.6..-1.1 ms per step; C2 (512 blocks, whose ragged last round the mixed
        // split already fills) +0.08 ms (profiles/flat_c2_ab.sh), so not there
        if (!noflat && Q >= 8192 && (flat_generic || ((const OrbitIndex *)ix->orbit)->gblk >= 1024)) {
            const int nb = (Q + 255) / 256;
            if ((size_t)Q > s.cap_flat) {
                if (s.fperm || s.fbcnt || s.fflag || s.fidx || s.ferr || s.ftile || s.fpal || s.fhm || s.fvm)
                    (void)hipDeviceSynchronize();  // (as above)
                dfree(s.fperm);
                dfree(s.fbcnt);
                dfree(s.fflag);
                dfree(s.fidx);
                dfree(s.ferr);
                dfree(s.ftile);
                dfree(s.fpal);
                dfree(s.fhm);
                dfree(s.fvm);
                s.fperm = s.fbcnt = s.fidx = nullptr;  // a failed allocation below leaves nothing dangling
                s.fflag = s.fhm = s.fvm = nullptr;
                s.ferr = nullptr;
                s.ftile = s.fpal = nullptr;
                s.cap_flat = 0;
                if (!s.fcnt) TILER_HIP_CHECK(dmalloc((void **)&s.fcnt, sizeof(int)));
                TILER_HIP_CHECK(dmalloc((void **)&s.fperm, (size_t)Q * sizeof(int)));
                TILER_HIP_CHECK(dmalloc((void **)&s.fbcnt, (size_t)nb * sizeof(int)));
                TILER_HIP_CHECK(dmalloc((void **)&s.fflag, (size_t)Q));
                TILER_HIP_CHECK(dmalloc((void **)&s.fidx, (size_t)Q * sizeof(int)));
                TILER_HIP_CHECK(dmalloc((void **)&s.ferr, (size_t)Q * sizeof(float)));
                TILER_HIP_CHECK(dmalloc((void **)&s.ftile, (size_t)Q * sizeof(int32_t)));
                TILER_HIP_CHECK(dmalloc((void **)&s.fpal, (size_t)Q * sizeof(int32_t)));
                TILER_HIP_CHECK(dmalloc((void **)&s.fhm, (size_t)Q));
                TILER_HIP_CHECK(dmalloc((void **)&s.fvm, (size_t)Q));
                s.cap_flat = Q;
            }
            hipLaunchKernelGGL(ft_flat_flag_kernel, dim3(nb), dim3(256), 0, stream, d_rgb, Q, s.fflag, s.fbcnt);
            hipLaunchKernelGGL(ft_flat_scan_kernel, dim3(1), dim3(1024), 0, stream, s.fbcnt, nb, s.fcnt);
            hipLaunchKernelGGL(ft_flat_place_kernel, dim3(nb), dim3(256), 0, stream, d_rgb, Q, (const uint8_t *)s.fflag,
                               (const int *)s.fbcnt, (const int *)s.fcnt, s.fperm);
            TILER_HIP_CHECK(hipGetLastError());
            FtMaps fm;
            if (maps) fm = FtMaps{s.ftile, s.fpal, s.fhm, s.fvm};
            ix->flat_cnt = s.fcnt;  // the shortlist reads the non-flat count on the device (no host sync)
            int rc = 0;
            if (flat_generic) {
                PsyvArgs pa;
                pa.n = Q;
                pa.rgb = d_rgb;
                pa.perm = s.fperm;
                pa.flags = PSYV_WAVELETS;
                pa.gamma = gamma;
                pa.out32 = s.qrows;
                if (fuse_rb) {
                    pa.box = ix->kd->d_box;
                    pa.rootbox = s.kd_rootbox;
                }
                rc = launch_psyv(pa, stream);
                if (!rc) rc = nn_search_dev(ix, s.qrows, Q, 1, s.fidx, s.ferr, maps ? &fm : nullptr, stream, fuse_rb);
            } else {
                rc = orbit_ft_queries(ix, d_rgb, Q, gamma, s.qrows, fuse_rb ? ix->kd->d_box : nullptr,
                                      fuse_rb ? s.kd_rootbox : nullptr, stream, s.fperm);
                if (!rc)
                    rc = nn_search_dev(ix, s.qrows, Q, 1, s.fidx, s.ferr, maps ? &fm : nullptr, stream, fuse_rb, true);
            }
            ix->flat_cnt = nullptr;
            if (rc) return -1;
            hipLaunchKernelGGL(ft_unpermute_kernel, dim3(nb), dim3(256), 0, stream, Q, (const int *)s.fperm,
                               (const int *)s.fidx, (const float *)s.ferr, (const int32_t *)s.ftile,
                               (const int32_t *)s.fpal, (const uint8_t *)s.fhm, (const uint8_t *)s.fvm, d_idx, d_err,
                               maps ? *maps : FtMaps{});
            TILER_HIP_CHECK(hipGetLastError());
            return 0;
        }
    }
    if (ix->orbit && use_wavelets) {
        // one kernel: descriptors + the orbit search's q' fragments and statistics (+ the kd root box)
        if (orbit_ft_queries(ix, d_rgb, Q, gamma, s.qrows, fuse_rb ? ix->kd->d_box : nullptr,
                             fuse_rb ? s.kd_rootbox : nullptr, stream))
            return -1;
        return nn_search_dev(ix, s.qrows, Q, 1, d_idx, d_err, maps, stream, fuse_rb, true);
    }
    PsyvArgs pa;
    pa.n = Q;
    pa.rgb = d_rgb;
    pa.flags = use_wavelets ? PSYV_WAVELETS : 0;
    pa.gamma = gamma;
    pa.out32 = s.qrows;
    if (fuse_rb) {  // annBoxDistance of each query descriptor, in the descriptor kernel (kd pruning check)
        pa.box = ix->kd->d_box;
        pa.rootbox = s.kd_rootbox;
    }
    if (launch_psyv(pa, stream)) return -1;
    return nn_search_dev(ix, s.qrows, Q, 1, d_idx, d_err, maps, stream, fuse_rb);
}

}  // namespace tiler

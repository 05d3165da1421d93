// kmodes.hip -- GlobalTiling K-Modes (TKModes, kmodes.pas:46-1060) on gfx950.
//
// Exact restatement of what the reference executes on x86-64 (asm dissimilarity kmodes.pas:316-596,
// 960-point snapshot bins, incremental modes, Delphi-LCG empty-cluster rescue), so labels and
// centroids are bit-identical to the CPU oracle (itself pinned against the reference asm).
// Byte work, no floating point: the dissimilarity is evaluated on packed dwords with v_sad_u8 (L1 of
// bytes 16..79) and a SWAR nonzero-byte count (mismatches), never reshaped into a GEMM.
//   dis = 2048 * #mismatch(80 B) + W0 + W4,  W0 = (|i8(r0-x0)| + 256|i8(r1-x1)| + S_lo) mod 2^16, ...
// Phases (ComputeKModes kmodes.pas:917-1060):
//   farthest-first init  : K rounds of {min-distance update + block argmax} / {select}   (698-776)
//   initial assignment   : all points vs K centroids, argmin ties -> last  (packed u64 atomicMin)
//   modes                : attribute histograms (atomics), first-max mode, RandInt rows for empties
//   KModesIter           : per 960-point bin: parallel assignment vs the CURRENT centroids, then one
//                          workgroup applies the bin's moves in order (MovePointCat over 80 lanes,
//                          rescue with a workgroup-parallel argmax and ordered member selection)
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "kmodes.hpp"

namespace tiler {

static constexpr int KM_A = 80;     // cKModesFeatureCount (kmodes.pas:15)
static constexpr int KM_BIN = 960;  // KModesIter cBinSize (kmodes.pas:847)

__device__ __forceinline__ unsigned abs_i8(unsigned r, unsigned x) {
    const int d = (int)(int8_t)(uint8_t)(r - x);  // psubb + pabsb
    return (unsigned)(d < 0 ? -d : d);
}

__device__ __forceinline__ unsigned nz_bytes(unsigned t) {  // number of non-zero bytes of t
    const unsigned m = (((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
    return __popc(m);
}

// row = list entry (centroid / member), x = item (kmodes.pas:341-412)
__device__ __forceinline__ unsigned long long km_dissim(const uint32_t *__restrict__ r, const uint32_t *__restrict__ x) {
    unsigned mism = 0, slo = 0, shi = 0;
#pragma unroll
    for (int w = 0; w < 20; w++) mism += nz_bytes(r[w] ^ x[w]);
#pragma unroll
    for (int w = 4; w < 20; w += 4) {
        slo = __builtin_amdgcn_sad_u8(r[w], x[w], slo);
        slo = __builtin_amdgcn_sad_u8(r[w + 1], x[w + 1], slo);
        shi = __builtin_amdgcn_sad_u8(r[w + 2], x[w + 2], shi);
        shi = __builtin_amdgcn_sad_u8(r[w + 3], x[w + 3], shi);
    }
    const unsigned r0 = r[0], x0 = x[0], r2 = r[2], x2 = x[2];
    const unsigned w0 = (abs_i8(r0 & 255, x0 & 255) + 256u * abs_i8((r0 >> 8) & 255, (x0 >> 8) & 255) + slo) & 0xffffu;
    const unsigned w4 = (abs_i8(r2 & 255, x2 & 255) + 256u * abs_i8((r2 >> 8) & 255, (x2 >> 8) & 255) + shi) & 0xffffu;
    return ((unsigned long long)mism << 11) + w0 + w4;
}

__device__ __forceinline__ void load_row(const uint8_t *__restrict__ p, uint32_t (&w)[20]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const uint4 v = q[i];
        w[4 * i] = v.x;
        w[4 * i + 1] = v.y;
        w[4 * i + 2] = v.z;
        w[4 * i + 3] = v.w;
    }
}

// RandInt kmodes.pas:82-86
__device__ __forceinline__ unsigned km_randint(unsigned range, unsigned *seed) {
    *seed = *seed * 0x08088405u + 1u;
    return (unsigned)(((unsigned long long)*seed * range) >> 32);
}

struct KmState {
    const uint8_t *X;  // [n][80], rows 16-byte aligned
    int n, K, M;
    int32_t *memb;
    uint8_t *cent;      // [K][80]
    int32_t *freq;      // [K][80][M]
    int32_t *csize;     // [K]
    unsigned long long *mind;  // [n]
    uint8_t *used;             // [n]
    unsigned long long *part;  // farthest-first partial argmax [nblk]
    int32_t *center;           // [K] chosen centre rows
    unsigned long long *akey;  // [n] packed (dis << 32) | ~idx for assignments
    unsigned *seed;
    unsigned long long *cost;  // [1]
    int *moves;                // [1]
    int *err;                  // [1]
};

// ---- farthest-first (InitFarthestFirst kmodes.pas:698-776) ----
// update mindist with the centre chosen last, then per-block argmax over unused points ('>=' -> last)
__global__ __launch_bounds__(256) void km_ff_update(KmState s, int j) {
    __shared__ unsigned long long best[256];
    const int c = s.center[j];
    uint32_t item[20];
    load_row(s.X + (long)c * KM_A, item);
    unsigned long long bk = 0;  // (value, index) max packed: value in high bits is not possible (u64 values)
    unsigned long long bv = 0;
    int bi = -1;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < s.n; i += (long)gridDim.x * 256) {
        uint32_t row[20];
        load_row(s.X + i * KM_A, row);
        const unsigned long long d = km_dissim(row, item);
        unsigned long long m = s.mind[i];
        if (d < m) {  // cmovb: strict-less (kmodes.pas:555-558); the 'used' skip is a no-op (567)
            m = d;
            s.mind[i] = m;
        }
        if (!s.used[i] && m >= bv) {  // ascending i within a thread: '>=' keeps the last
            bv = m;
            bi = (int)i;
        }
    }
    (void)bk;
    // block reduce (value max, ties -> larger index); value fits 32 bits (dis < 2^19) unless UINT64_MAX
    const unsigned long long v32 = bv > 0xFFFFFFFFull ? 0xFFFFFFFFull : bv;
    best[threadIdx.x] = (bi < 0) ? 0ull : ((v32 << 32) | (unsigned)(bi + 1));
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) best[threadIdx.x] = max(best[threadIdx.x], best[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) s.part[blockIdx.x] = best[0];
}

__global__ __launch_bounds__(256) void km_ff_select(KmState s, int j, int nblk) {
    __shared__ unsigned long long best[256];
    unsigned long long b = 0;
    for (int i = threadIdx.x; i < nblk; i += 256) b = max(b, s.part[i]);
    best[threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) best[threadIdx.x] = max(best[threadIdx.x], best[threadIdx.x + o]);
        __syncthreads();
    }
    const unsigned long long w = best[0];
    const int f = (w == 0) ? -1 : (int)(w & 0xFFFFFFFFull) - 1;
    if (f < 0) {
        if (threadIdx.x == 0) *s.err = 1;
        return;
    }
    if (threadIdx.x < KM_A) s.cent[(long)j * KM_A + threadIdx.x] = s.X[(long)f * KM_A + threadIdx.x];
    if (threadIdx.x == 0) {
        s.center[j] = f;
        s.used[f] = 1;
    }
}

// ---- assignment: akey[i] = min over centroids of (dis << 32 | ~c)  (argmin, ties -> last centroid) ----
// grid: (points / 256, centroid splits); centroids staged through LDS in tiles of 128
__global__ __launch_bounds__(256) void km_assign(KmState s, int p0, int p1, int csplit) {
    __shared__ uint4 ct[128 * 5];
    const long i = p0 + (long)blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < p1;
    uint32_t item[20];
    if (valid) load_row(s.X + i * KM_A, item);
    const int per = (s.K + csplit - 1) / csplit;
    const int c0 = blockIdx.y * per, c1 = min(s.K, c0 + per);
    unsigned long long best = ~0ull;
    for (int t0 = c0; t0 < c1; t0 += 128) {
        const int cnt = min(128, c1 - t0);
        __syncthreads();
        for (int e = threadIdx.x; e < cnt * 5; e += 256)
            ct[e] = reinterpret_cast<const uint4 *>(s.cent + (long)t0 * KM_A)[e];
        __syncthreads();
        if (valid) {
            for (int c = 0; c < cnt; c++) {
                uint32_t row[20];
#pragma unroll
                for (int q = 0; q < 5; q++) {
                    const uint4 v = ct[c * 5 + q];
                    row[4 * q] = v.x;
                    row[4 * q + 1] = v.y;
                    row[4 * q + 2] = v.z;
                    row[4 * q + 3] = v.w;
                }
                const unsigned long long d = km_dissim(row, item);
                const unsigned long long key = (d << 32) | (0xFFFFFFFFu - (unsigned)(t0 + c));
                best = key < best ? key : best;
            }
        }
    }
    if (valid) atomicMin(&s.akey[i], best);
}

__global__ void km_fill_u64(unsigned long long *p, long n, unsigned long long v) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = v;
}

// initial labels + histograms (ComputeKModes kmodes.pas:984-1008)
__global__ __launch_bounds__(256) void km_init_hist(KmState s) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < s.n; i += (long)gridDim.x * 256) {
        const int c = (int)(0xFFFFFFFFu - (unsigned)(s.akey[i] & 0xFFFFFFFFull));
        s.memb[i] = c;
        atomicAdd(&s.csize[c], 1);
        for (int a = 0; a < KM_A; a++) atomicAdd(&s.freq[((long)c * KM_A + a) * s.M + s.X[i * KM_A + a]], 1);
    }
}

// modes (kmodes.pas:1010-1021): empty clusters take X[RandInt(n)][a] per attribute in (k, a) order
__global__ __launch_bounds__(256) void km_init_modes(KmState s, int32_t *rand_rows) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned seed = *s.seed;
        for (int k = 0; k < s.K; k++)
            if (s.csize[k] == 0)
                for (int a = 0; a < KM_A; a++) rand_rows[(long)k * KM_A + a] = (int)km_randint((unsigned)s.n, &seed);
        *s.seed = seed;
    }
}

__global__ __launch_bounds__(256) void km_init_modes2(KmState s, const int32_t *rand_rows) {
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < (long)s.K * KM_A; e += (long)gridDim.x * 256) {
        const int k = (int)(e / KM_A), a = (int)(e % KM_A);
        if (s.csize[k] == 0) {
            s.cent[e] = s.X[(long)rand_rows[e] * KM_A + a];
        } else {
            const int32_t *f = s.freq + e * s.M;
            int bi = -1, bv = INT32_MIN;
            for (int m = 0; m < s.M; m++)
                if (f[m] > bv) {
                    bv = f[m];
                    bi = m;
                }
            s.cent[e] = (uint8_t)bi;  // GetMaxValueIndex: first max (kmodes.pas:149-161)
        }
    }
}

// ---- the sequential part of one bin (KModesIter kmodes.pas:869-911), one workgroup of 128 ----
__device__ void move_point_cat(const KmState &s, int ip, int to, int from) {
    // lanes = attributes (MovePointCat kmodes.pas:778-806); caller syncs around
    const int a = threadIdx.x;
    if (a < KM_A) {
        const int cur = s.X[(long)ip * KM_A + a];
        int32_t *tc = s.freq + ((long)to * KM_A + a) * s.M;
        int32_t *fc = s.freq + ((long)from * KM_A + a) * s.M;
        tc[cur]++;
        uint8_t *ct = s.cent + (long)to * KM_A + a;
        if (tc[*ct] < tc[cur]) *ct = (uint8_t)cur;
        fc[cur]--;
        uint8_t *cf = s.cent + (long)from * KM_A + a;
        if (*cf == cur) {
            int bi = -1, bv = INT32_MIN;
            for (int m = 0; m < s.M; m++)
                if (fc[m] > bv) {
                    bv = fc[m];
                    bi = m;
                }
            *cf = (uint8_t)bi;
        }
    }
    if (threadIdx.x == 0) {
        s.memb[ip] = to;
        s.csize[to]++;
        s.csize[from]--;
    }
}

__global__ __launch_bounds__(128) void km_bin_seq(KmState s, int p0, int p1) {
    __shared__ int sh_i[4];
    __shared__ unsigned long long sh_best[128];
    __shared__ int sh_cnt[128];
    unsigned long long cost = 0;
    int moves = 0;
    for (int i = p0; i < p1; i++) {
        const unsigned long long key = s.akey[i];
        const int cl = (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
        cost += key >> 32;
        const int old = s.memb[i];
        if (old == cl) continue;  // uniform
        moves++;
        __syncthreads();
        move_point_cat(s, i, cl, old);
        __syncthreads();
        if (s.csize[old] != 0) continue;
        // GetMaxClusterMembers (kmodes.pas:631-669): largest cluster, ties -> last
        unsigned long long b = 0;
        for (int c = threadIdx.x; c < s.K; c += 128) {
            const unsigned long long v = ((unsigned long long)(unsigned)s.csize[c] << 32) | (unsigned)c;
            b = v > b ? v : b;
        }
        sh_best[threadIdx.x] = b;
        __syncthreads();
        for (int o = 64; o > 0; o >>= 1) {
            if (threadIdx.x < o) sh_best[threadIdx.x] = max(sh_best[threadIdx.x], sh_best[threadIdx.x + o]);
            __syncthreads();
        }
        const int from = (int)(sh_best[0] & 0xFFFFFFFFull);
        const int cnt = s.csize[from];
        if (threadIdx.x == 0) sh_i[0] = (int)km_randint((unsigned)cnt, s.seed);
        __syncthreads();
        const int r = sh_i[0];
        // r-th member of 'from' in ascending point order (choices[RandInt(cnt)], kmodes.pas:895-902)
        const long chunk = (s.n + 127) / 128;
        const long a0 = threadIdx.x * chunk, a1 = min((long)s.n, a0 + chunk);
        int mine = 0;
        for (long q = a0; q < a1; q++) mine += s.memb[q] == from;
        sh_cnt[threadIdx.x] = mine;
        __syncthreads();
        if (threadIdx.x == 0) {
            int acc = 0, t = 0;
            while (t < 128 && acc + sh_cnt[t] <= r) acc += sh_cnt[t++];
            sh_i[1] = t;
            sh_i[2] = r - acc;
        }
        __syncthreads();
        if (threadIdx.x == sh_i[1]) {
            int left = sh_i[2];
            for (long q = a0; q < a1; q++)
                if (s.memb[q] == from && left-- == 0) {
                    sh_i[3] = (int)q;
                    break;
                }
        }
        __syncthreads();
        move_point_cat(s, sh_i[3], old, from);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        s.cost[0] += cost;
        s.moves[0] += moves;
    }
}

static int km_run(KmState &s, int start, int *n_iter, unsigned long long *cost_out, hipStream_t st) {
    const int n = s.n, K = s.K;
    const int nblk_ff = std::min(1024, (n + 255) / 256);
    // InitFarthestFirst
    hipLaunchKernelGGL(km_fill_u64, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, st, s.mind, (long)n, ~0ull);
    TILER_HIP_CHECK(hipMemsetAsync(s.used, 0, n, st));
    TILER_HIP_CHECK(hipMemsetAsync(s.cent, 0xff, (size_t)K * KM_A, st));
    TILER_HIP_CHECK(hipMemcpyAsync(s.center, &start, sizeof(int), hipMemcpyHostToDevice, st));
    TILER_HIP_CHECK(hipMemcpyAsync(s.cent, s.X + (long)start * KM_A, KM_A, hipMemcpyDeviceToDevice, st));
    {
        const uint8_t one = 1;
        TILER_HIP_CHECK(hipMemcpyAsync(s.used + start, &one, 1, hipMemcpyHostToDevice, st));
    }
    {
        KTimer tm("kmodes_init", st);
        for (int j = 0; j < K; j++) {
            hipLaunchKernelGGL(km_ff_update, dim3(nblk_ff), dim3(256), 0, st, s, j);
            if (j + 1 < K) hipLaunchKernelGGL(km_ff_select, dim3(1), dim3(256), 0, st, s, j + 1, nblk_ff);
        }
    }
    TILER_HIP_CHECK(hipGetLastError());
    // initial assignment + modes
    const int csplit = std::max(1, std::min(64, (K + 511) / 512));
    hipLaunchKernelGGL(km_fill_u64, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, st, s.akey, (long)n, ~0ull);
    {
        KTimer tm("kmodes_assign", st);
        hipLaunchKernelGGL(km_assign, dim3((n + 255) / 256, csplit), dim3(256), 0, st, s, 0, n, csplit);
    }
    TILER_HIP_CHECK(hipMemsetAsync(s.csize, 0, (size_t)K * 4, st));
    TILER_HIP_CHECK(hipMemsetAsync(s.freq, 0, (size_t)K * KM_A * s.M * 4, st));
    hipLaunchKernelGGL(km_init_hist, dim3(std::min(2048, (n + 255) / 256)), dim3(256), 0, st, s);
    int32_t *rand_rows = nullptr;
    TILER_HIP_CHECK(hipMallocAsync((void **)&rand_rows, (size_t)K * KM_A * 4, st));
    hipLaunchKernelGGL(km_init_modes, dim3(1), dim3(64), 0, st, s, rand_rows);
    hipLaunchKernelGGL(km_init_modes2, dim3(std::min(4096, (K * KM_A + 255) / 256)), dim3(256), 0, st, s, rand_rows);
    TILER_HIP_CHECK(hipFreeAsync(rand_rows, st));
    TILER_HIP_CHECK(hipGetLastError());
    // iterations (kmodes.pas:1023-1039)
    unsigned long long cost = ~0ull;
    int itr = 0;
    struct {
        unsigned long long cost;
        int moves;
        int err;
    } h;
    for (;;) {
        itr++;
        TILER_HIP_CHECK(hipMemsetAsync(s.cost, 0, 8, st));
        TILER_HIP_CHECK(hipMemsetAsync(s.moves, 0, 4, st));
        for (int b0 = 0; b0 < n; b0 += KM_BIN) {
            const int b1 = std::min(n, b0 + KM_BIN);
            hipLaunchKernelGGL(km_fill_u64, dim3((b1 - b0 + 255) / 256), dim3(256), 0, st, s.akey + b0, (long)(b1 - b0),
                               ~0ull);
            {
                KTimer tm("kmodes_assign", st);
                hipLaunchKernelGGL(km_assign, dim3((b1 - b0 + 255) / 256, csplit), dim3(256), 0, st, s, b0, b1, csplit);
            }
            {
                KTimer tm("kmodes_seq", st);
                hipLaunchKernelGGL(km_bin_seq, dim3(1), dim3(128), 0, st, s, b0, b1);
            }
        }
        TILER_HIP_CHECK(hipGetLastError());
        TILER_HIP_CHECK(hipMemcpyAsync(&h.cost, s.cost, 8, hipMemcpyDeviceToHost, st));
        TILER_HIP_CHECK(hipMemcpyAsync(&h.moves, s.moves, 4, hipMemcpyDeviceToHost, st));
        TILER_HIP_CHECK(hipMemcpyAsync(&h.err, s.err, 4, hipMemcpyDeviceToHost, st));
        TILER_HIP_CHECK(hipStreamSynchronize(st));
        if (h.err) {
            set_error("kmodes: farthest-first ran out of points (k > n)");
            return -1;
        }
        const bool conv = (h.cost >= cost) || (h.moves == 0);
        cost = h.cost;
        if (conv) break;
    }
    if (n_iter) *n_iter = itr;
    if (cost_out) *cost_out = cost;
    return 0;
}

int kmodes_compute_dev(const uint8_t *d_X, int n, int k, int start_point, int n_modalities, int32_t *d_labels,
                       uint8_t *d_centroids, int *n_iter, uint64_t *cost, hipStream_t st) {
    if (n <= 0 || k <= 0 || k > n || start_point < 0 || start_point >= n || n_modalities <= 0 || n_modalities > 256) {
        set_error("kmodes: invalid arguments (need 0 < k <= n, 0 <= start < n, 0 < modalities <= 256)");
        return -1;
    }
    if (((uintptr_t)d_X & 15) != 0) {
        set_error("kmodes: X must be 16-byte aligned");
        return -1;
    }
    KmState s{};
    s.X = d_X;
    s.n = n;
    s.K = k;
    s.M = n_modalities;
    s.memb = d_labels;
    // centroid storage must be 16-byte aligned rows of 80 B: use a private buffer
    char *buf = nullptr;
    const int nblk_ff = std::min(1024, (n + 255) / 256);
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_cent = carve((size_t)k * KM_A), o_freq = carve((size_t)k * KM_A * n_modalities * 4),
                 o_csize = carve((size_t)k * 4), o_mind = carve((size_t)n * 8), o_used = carve(n),
                 o_part = carve((size_t)nblk_ff * 8), o_center = carve((size_t)k * 4), o_akey = carve((size_t)n * 8),
                 o_misc = carve(64);
    TILER_HIP_CHECK(hipMalloc((void **)&buf, off));
    s.cent = (uint8_t *)(buf + o_cent);
    s.freq = (int32_t *)(buf + o_freq);
    s.csize = (int32_t *)(buf + o_csize);
    s.mind = (unsigned long long *)(buf + o_mind);
    s.used = (uint8_t *)(buf + o_used);
    s.part = (unsigned long long *)(buf + o_part);
    s.center = (int32_t *)(buf + o_center);
    s.akey = (unsigned long long *)(buf + o_akey);
    s.seed = (unsigned *)(buf + o_misc);
    s.cost = (unsigned long long *)(buf + o_misc + 8);
    s.moves = (int *)(buf + o_misc + 16);
    s.err = (int *)(buf + o_misc + 20);
    const unsigned seed0 = 0x42381337u;  // ComputeKModes kmodes.pas:930
    int rc = -1;
    do {
        if (hipMemsetAsync(buf + o_misc, 0, 64, st) != hipSuccess) break;
        if (hipMemcpyAsync(s.seed, &seed0, 4, hipMemcpyHostToDevice, st) != hipSuccess) break;
        unsigned long long c = 0;
        if (km_run(s, start_point, n_iter, &c, st)) break;
        if (cost) *cost = c;
        if (hipMemcpyAsync(d_centroids, s.cent, (size_t)k * KM_A, hipMemcpyDeviceToDevice, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        rc = 0;
    } while (0);
    (void)hipFree(buf);
    return rc;
}

// ---- DoKModes medoid choice (main.pas:4231-4253): per cluster j with members, the member minimising
// dissim(member, centroid_j) (GetMinMatchingDissim(ToMerge, LocCentroids[j]) -> ties: last member) ----
__global__ __launch_bounds__(256) void km_medoid_kernel(const uint8_t *X, int n, const int32_t *labels,
                                                        const uint8_t *cent, unsigned long long *best,
                                                        int32_t *counts) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const int j = labels[i];
        uint32_t row[20], item[20];
        load_row(X + i * KM_A, row);
        load_row(cent + (long)j * KM_A, item);
        const unsigned long long d = km_dissim(row, item);
        atomicMin(&best[j], (d << 32) | (0xFFFFFFFFu - (unsigned)i));
        atomicAdd(&counts[j], 1);
    }
}

int kmodes_medoids_host(const uint8_t *X, int n, const int32_t *labels, const uint8_t *centroids, int k,
                        int32_t *medoid, int32_t *counts) {
    if (n < 0 || k <= 0 || (n > 0 && (!X || !labels)) || !centroids || !medoid || !counts) {
        set_error("kmodes_medoids: invalid arguments");
        return -1;
    }
    for (int i = 0; i < n; i++)
        if (labels[i] < 0 || labels[i] >= k) {
            set_error("kmodes_medoids: label out of range");
            return -1;
        }
    char *buf = nullptr;
    const size_t oX = 0, oL = ((size_t)n * KM_A + 255) & ~(size_t)255, oC = oL + (((size_t)n * 4 + 255) & ~(size_t)255),
                 oB = oC + (((size_t)k * KM_A + 255) & ~(size_t)255), oN = oB + (size_t)k * 8, total = oN + (size_t)k * 4;
    TILER_HIP_CHECK(hipMalloc((void **)&buf, total));
    int rc = -1;
    do {
        if (n > 0 && hipMemcpy(buf + oX, X, (size_t)n * KM_A, hipMemcpyHostToDevice) != hipSuccess) break;
        if (n > 0 && hipMemcpy(buf + oL, labels, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) break;
        if (hipMemcpy(buf + oC, centroids, (size_t)k * KM_A, hipMemcpyHostToDevice) != hipSuccess) break;
        if (hipMemset(buf + oB, 0xff, (size_t)k * 8) != hipSuccess) break;
        if (hipMemset(buf + oN, 0, (size_t)k * 4) != hipSuccess) break;
        if (n > 0)
            hipLaunchKernelGGL(km_medoid_kernel, dim3(std::min(4096, (n + 255) / 256)), dim3(256), 0, nullptr,
                               (const uint8_t *)(buf + oX), n, (const int32_t *)(buf + oL),
                               (const uint8_t *)(buf + oC), (unsigned long long *)(buf + oB), (int32_t *)(buf + oN));
        if (hipGetLastError() != hipSuccess) break;
        std::vector<unsigned long long> b(k);
        if (hipMemcpy(b.data(), buf + oB, (size_t)k * 8, hipMemcpyDeviceToHost) != hipSuccess) break;
        if (hipMemcpy(counts, buf + oN, (size_t)k * 4, hipMemcpyDeviceToHost) != hipSuccess) break;
        for (int j = 0; j < k; j++)
            medoid[j] = counts[j] > 0 ? (int32_t)(0xFFFFFFFFu - (unsigned)(b[j] & 0xFFFFFFFFull)) : -1;
        rc = 0;
    } while (0);
    if (rc) set_error("kmodes_medoids: HIP failure");
    (void)hipFree(buf);
    return rc;
}

int kmodes_compute_host(const uint8_t *X, int n, int nattr, int k, int start_point, int n_modalities,
                        int32_t *labels, uint8_t *centroids, int *n_iter, uint64_t *cost) {
    if (nattr != KM_A) {
        set_error("kmodes: nattr must be 80 (cKModesFeatureCount; the asm dissimilarity is 80-byte wide)");
        return -1;
    }
    if (!X || !labels || !centroids) {
        set_error("kmodes: null buffer");
        return -1;
    }
    uint8_t *d_X = nullptr, *d_c = nullptr;
    int32_t *d_l = nullptr;
    hipStream_t st = nullptr;
    TILER_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int rc = -1;
    do {
        if (hipMalloc((void **)&d_X, (size_t)std::max(n, 1) * KM_A) != hipSuccess) break;
        if (hipMalloc((void **)&d_c, (size_t)std::max(k, 1) * KM_A) != hipSuccess) break;
        if (hipMalloc((void **)&d_l, (size_t)std::max(n, 1) * 4) != hipSuccess) break;
        if (n > 0 && hipMemcpyAsync(d_X, X, (size_t)n * KM_A, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (kmodes_compute_dev(d_X, n, k, start_point, n_modalities, d_l, d_c, n_iter, cost, st)) {
            rc = -2;
            break;
        }
        if (hipMemcpyAsync(labels, d_l, (size_t)n * 4, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(centroids, d_c, (size_t)k * KM_A, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        rc = k;
    } while (0);
    if (rc == -1) set_error("kmodes: HIP failure");
    (void)hipFree(d_X);
    (void)hipFree(d_c);
    (void)hipFree(d_l);
    (void)hipStreamDestroy(st);
    return rc < 0 ? -1 : rc;
}

}  // namespace tiler

// kmeans.hip -- the k-means of the Dither step on the GPU (PrepareDitherTiles main.pas:2097-2152: yakmo_create(
// FPaletteCount, 1 restart, MaxInt iterations, k-means++ init, seed 0, no normalisation) over the keyframe's LAB +
// wavelet descriptors -> DitheringPalIndex (the labels) and PaletteCentroids).
//
// yakmo.dll ships as a binary only, so the algorithm is its published one, written down exactly (the
// CPU restatement oracle/kmeans.c follows the same text, and parity with the DLL is unpinned):
//   * distances: sum over d ascending of (x_d - c_d)^2 in fp64, no contraction; ties -> the lowest centroid;
//   * k-means++ seeding from MT19937(seed) uniforms u = genrand_int32 / 2^32: the first centre is point
//     floor(u * n); each next one is drawn with probability D(x)^2 / sum D^2 -- the sum over runs of
//     L = ceil(n / 1024) consecutive points (sequential inside a run, then the run sums in order), the pick the
//     first point whose running sum exceeds u * sum (floor(u * n) when the sum is 0);
//   * Lloyd iterations until no label changes (or max_iter assignments): a centroid is the mean of its members in
//     point order, summed in runs of 256 members (sequential inside a run, run sums in order) and divided by the
//     count; an empty cluster keeps its centroid.
// Layout: X [n][d] row-major (centroid means, seeding rows); X^T [d][n] for the per-point distances of the seeding
// and the assignment (lane = point, coalesced).
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "kmeans.hpp"
#include "psyv.hpp"
#include "tiler_common.hpp"

#pragma clang fp contract(off)

namespace tiler {

namespace {

constexpr int KM_MAXD = 192;    // descriptor dimension bound (cTileDCTSize)
constexpr int KM_CH = 32;       // centroids per LDS chunk of the assignment (distance chains per lane)
constexpr int KM_RUN = 256;     // members per centroid partial sum
constexpr int KM_SEL_T = 1024;  // seeding selection workgroup

// MT19937 (Matsumoto & Nishimura), init_genrand / genrand_int32
struct Mt19937 {
    uint32_t mt[624];
    int mti;
    explicit Mt19937(uint32_t s) {
        mt[0] = s;
        for (mti = 1; mti < 624; mti++) mt[mti] = 1812433253u * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
    }
    uint32_t next() {
        if (mti >= 624) {
            for (int kk = 0; kk < 624; kk++) {
                const uint32_t y = (mt[kk] & 0x80000000u) | (mt[(kk + 1) % 624] & 0x7fffffffu);
                mt[kk] = mt[(kk + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            mti = 0;
        }
        uint32_t y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    double uniform() { return (double)next() * (1.0 / 4294967296.0); }
};

__global__ __launch_bounds__(256) void km_transpose_kernel(const double *__restrict__ X, long n, int d,
                                                           double *__restrict__ XT) {
    __shared__ double tile[32][33];
    const long i0 = (long)blockIdx.x * 32;
    const int d0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int r = ty; r < 32; r += 8) {
        const long i = i0 + r;
        const int dd = d0 + tx;
        tile[r][tx] = (i < n && dd < d) ? X[i * d + dd] : 0.0;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int dd = d0 + r;
        const long i = i0 + tx;
        if (dd < d && i < n) XT[(long)dd * n + i] = tile[tx][r];
    }
}

// mind2[i] = min(mind2[i], |x_i - c|^2) (first centre: assignment); lane = point, X^T coalesced
__global__ __launch_bounds__(256) void km_mind_kernel(const double *__restrict__ XT, long n, int d,
                                                      const double *__restrict__ c, double *__restrict__ mind2,
                                                      int first) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double acc = 0.0;
    for (int k = 0; k < d; k++) {
        const double t = XT[(long)k * n + i] - c[k];
        acc = acc + t * t;
    }
    mind2[i] = first ? acc : (acc < mind2[i] ? acc : mind2[i]);
}

// k-means++ draw s: the blocked sum of mind2, the pick, the new centre's row -> cent[s]
__global__ __launch_bounds__(KM_SEL_T) void km_select_kernel(const double *__restrict__ X, long n, int d,
                                                             const double *__restrict__ mind2,
                                                             const double *__restrict__ u, int s,
                                                             double *__restrict__ cent, long *__restrict__ pick_out) {
    __shared__ double part[KM_SEL_T];
    __shared__ long pick;
    const int t = threadIdx.x;
    const long L = (n + KM_SEL_T - 1) / KM_SEL_T;
    const long b = (long)t * L, e = b + L < n ? b + L : n;
    double acc = 0.0;
    for (long i = b; i < e; i++) acc = acc + mind2[i];
    part[t] = acc;
    __syncthreads();
    if (t == 0) {
        double S = 0.0;
        for (int r = 0; r < KM_SEL_T; r++) S = S + part[r];
        const double uu = u[s];
        long p = -1;
        if (S > 0.0) {
            const double target = uu * S;
            double run = 0.0;
            for (int r = 0; r < KM_SEL_T && p < 0; r++) {
                if (run + part[r] > target) {
                    const long rb = (long)r * L, re = rb + L < n ? rb + L : n;
                    double a2 = run;
                    for (long i = rb; i < re; i++) {
                        a2 = a2 + mind2[i];
                        if (a2 > target) {
                            p = i;
                            break;
                        }
                    }
                    if (p < 0) p = re - 1;
                } else {
                    run = run + part[r];
                }
            }
            if (p < 0) p = n - 1;
        } else {
            p = (long)(uu * (double)n);
            if (p >= n) p = n - 1;
        }
        pick = p;
        pick_out[s] = p;
    }
    __syncthreads();
    for (int k = t; k < d; k += KM_SEL_T) cent[(long)s * d + k] = X[pick * d + k];
}

__global__ __launch_bounds__(256) void km_copy_row_kernel(const double *__restrict__ X, int d, long row,
                                                          double *__restrict__ dst) {
    for (int k = threadIdx.x; k < d; k += 256) dst[k] = X[row * d + k];
}

// Lloyd assignment: lane = point (X^T [d][n]: one coalesced load per dimension), the centroids KM_CH at a time
// through LDS as [d][KM_CH] (each read a broadcast of two centroids' values), every lane keeping KM_CH distance
// chains in dimension order; the first minimum over chunks, then over a chunk's centroids in index order (ties ->
// the lowest centroid).  Per (dimension, centroid): sub, mul, add in fp64 (no contraction) -- the bound is the fp64
// VALU rate; per dimension a lane issues 3 * KM_CH of them against KM_CH / 2 LDS reads and one global load.
__global__ __launch_bounds__(256) void km_assign_kernel(const double *__restrict__ XT, long n, int d,
                                                        const double *__restrict__ cent, int k,
                                                        int32_t *__restrict__ labels, int *__restrict__ changed) {
    __shared__ double2 sc[KM_MAXD * KM_CH / 2];  // sc[dd * KM_CH / 2 + jp] = (c[2 jp][dd], c[2 jp + 1][dd])
    const long p = (long)blockIdx.x * 256 + threadIdx.x;
    const long pc = p < n ? p : n - 1;
    double best = HUGE_VAL;
    int bc = -1;
    for (int c0 = 0; c0 < k; c0 += KM_CH) {
        const int nc = k - c0 < KM_CH ? k - c0 : KM_CH;
        __syncthreads();
        for (int idx = threadIdx.x; idx < d * KM_CH; idx += 256) {
            const int dd = idx / KM_CH, cc = idx % KM_CH;
            reinterpret_cast<double *>(sc)[idx] = cc < nc ? cent[(long)(c0 + cc) * d + dd] : 0.0;
        }
        __syncthreads();
        double acc[KM_CH];
#pragma unroll
        for (int j = 0; j < KM_CH; j++) acc[j] = 0.0;
        double x = XT[pc];
        for (int dd = 0; dd < d; dd++) {
            const double xn = XT[(long)(dd + 1 < d ? dd + 1 : dd) * n + pc];  // the next dimension in flight
#pragma unroll
            for (int jp = 0; jp < KM_CH / 2; jp++) {
                const double2 cv = sc[dd * (KM_CH / 2) + jp];
                const double t0 = x - cv.x, t1 = x - cv.y;
                acc[2 * jp] = acc[2 * jp] + t0 * t0;
                acc[2 * jp + 1] = acc[2 * jp + 1] + t1 * t1;
            }
            x = xn;
        }
#pragma unroll
        for (int j = 0; j < KM_CH; j++)
            if (j < nc && acc[j] < best) {
                best = acc[j];
                bc = c0 + j;
            }
    }
    const bool ch = p < n && labels[p] != bc;
    if (ch) labels[p] = bc;
    const unsigned long long m = __ballot(ch);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(changed, (int)__popcll(m));
}

__global__ void km_iota_kernel(int32_t *v, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) v[i] = (int32_t)i;
}

// member counts per cluster from the label-sorted keys: seg[c] = lower bound of c
__global__ void km_seg_kernel(const uint32_t *__restrict__ sorted_labels, long n, int k, int *__restrict__ seg) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c > k) return;
    long lo = 0, hi = n;
    while (lo < hi) {
        const long mid = (lo + hi) >> 1;
        if (sorted_labels[mid] < (uint32_t)c)
            lo = mid + 1;
        else
            hi = mid;
    }
    seg[c] = (int)lo;
}

// one run of <= KM_RUN members of one cluster: partial[run][t] (thread = dimension)
__global__ __launch_bounds__(256) void km_partial_kernel(const double *__restrict__ X, int d,
                                                         const int32_t *__restrict__ members,
                                                         const int *__restrict__ run_first,
                                                         const int *__restrict__ run_count,
                                                         double *__restrict__ partial) {
    const int r = blockIdx.x;
    const int b = run_first[r], m = run_count[r];
    for (int t = threadIdx.x; t < d; t += 256) {
        double acc = 0.0;
        for (int i = 0; i < m; i++) acc = acc + X[(long)members[b + i] * d + t];
        partial[(long)r * d + t] = acc;
    }
}

__global__ __launch_bounds__(256) void km_mean_kernel(const double *__restrict__ partial, int d, int k,
                                                      const int *__restrict__ crun, const int *__restrict__ seg,
                                                      double *__restrict__ cent) {
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)k * d) return;
    const int c = (int)(idx / d), t = (int)(idx % d);
    const int cnt = seg[c + 1] - seg[c];
    if (cnt == 0) return;  // empty: the centroid stays
    double acc = 0.0;
    for (int r = crun[c]; r < crun[c + 1]; r++) acc = acc + partial[(long)r * d + t];
    cent[idx] = acc / (double)cnt;
}

}  // namespace

int kmeans_dev(const double *d_X, long n, int d, int k, int max_iter, uint32_t seed, int32_t *d_labels, double *d_cent,
               int *iterations, hipStream_t stream) {
    if (n <= 0 || d <= 0 || d > KM_MAXD || k <= 0 || !d_X || !d_labels || !d_cent || max_iter <= 0 ||
        n > 0x7fffffffL) {
        set_error("kmeans: invalid arguments (1 <= d <= 192, k >= 1, n >= 1)");
        return -1;
    }
    // RNG stream of the seeding (host): k uniforms
    Mt19937 rng(seed);
    std::vector<double> us(k);
    for (int s = 0; s < k; s++) us[s] = rng.uniform();
    const size_t nn = (size_t)n;
    size_t tmp_sort = 0;
    TILER_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, (const uint32_t *)nullptr,
                                                       (uint32_t *)nullptr, (const int32_t *)nullptr, (int32_t *)nullptr,
                                                       (int)n, 0, 32, stream));
    const long max_runs = n / KM_RUN + k + 1;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bytes = al(8 * nn * d) /* XT */ + al(8 * nn) /* mind2 */ + al(8 * (size_t)k) + al(8 * (size_t)k) +
                         2 * al(4 * nn) /* sort keys */ + 2 * al(4 * nn) /* sort values */ + al(tmp_sort) +
                         al(4 * (size_t)(k + 2)) * 2 + al(4 * (size_t)max_runs) * 2 + al(8 * (size_t)max_runs * d) +
                         al(4 * 4) + 1024;
    char *ws = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&ws, bytes));
    char *cur = ws;
    auto take = [&](size_t b) {
        char *r = cur;
        cur += al(b);
        return r;
    };
    double *XT = (double *)take(8 * nn * d);
    double *mind2 = (double *)take(8 * nn);
    double *d_u = (double *)take(8 * (size_t)k);
    long *d_pick = (long *)take(8 * (size_t)k);
    uint32_t *sk0 = (uint32_t *)take(4 * nn), *sk1 = (uint32_t *)take(4 * nn);
    int32_t *sv0 = (int32_t *)take(4 * nn), *sv1 = (int32_t *)take(4 * nn);
    void *tmp = take(tmp_sort);
    int *d_seg = (int *)take(4 * (size_t)(k + 2));
    int *d_crun = (int *)take(4 * (size_t)(k + 2));
    int *d_rfirst = (int *)take(4 * (size_t)max_runs);
    int *d_rcount = (int *)take(4 * (size_t)max_runs);
    double *partial = (double *)take(8 * (size_t)max_runs * d);
    int *d_changed = (int *)take(16);
    int rc = -1, it = 0;
    std::vector<int> seg(k + 1), crun(k + 1), rfirst, rcount;
    do {
        KTimer tt("kmeans", stream);
        if (hipMemcpyAsync(d_u, us.data(), 8 * (size_t)k, hipMemcpyHostToDevice, stream) != hipSuccess) break;
        hipLaunchKernelGGL(km_transpose_kernel, dim3((unsigned)((n + 31) / 32), (unsigned)((d + 31) / 32)), dim3(256), 0,
                           stream, d_X, n, d, XT);
        // k-means++ seeding
        long first = (long)(us[0] * (double)n);
        if (first >= n) first = n - 1;
        hipLaunchKernelGGL(km_copy_row_kernel, dim3(1), dim3(256), 0, stream, d_X, d, first, d_cent);
        bool ok = hipGetLastError() == hipSuccess;
        for (int s = 1; s < k && ok; s++) {
            hipLaunchKernelGGL(km_mind_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, XT, n, d,
                               d_cent + (long)(s - 1) * d, mind2, s == 1 ? 1 : 0);
            hipLaunchKernelGGL(km_select_kernel, dim3(1), dim3(KM_SEL_T), 0, stream, d_X, n, d, mind2, d_u, s, d_cent,
                               d_pick);
            ok = hipGetLastError() == hipSuccess;
        }
        if (!ok) break;
        if (hipMemsetAsync(d_labels, 0xff, 4 * nn, stream) != hipSuccess) break;  // -1: every first label changes
        const unsigned g_assign = (unsigned)((n + 255) / 256);
        bool fail = false;
        while (it < max_iter) {
            {
                KTimer ta("kmeans_assign", stream);
                if (hipMemsetAsync(d_changed, 0, 4, stream) != hipSuccess) {
                    fail = true;
                    break;
                }
                hipLaunchKernelGGL(km_assign_kernel, dim3(g_assign), dim3(256), 0, stream, XT, n, d, d_cent, k, d_labels,
                                   d_changed);
            }
            int changed = 0;
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(&changed, d_changed, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess) {
                fail = true;
                break;
            }
            it++;
            if (changed == 0 || it >= max_iter) break;
            // update: members sorted by (label, point) -> runs of KM_RUN -> partial sums -> means
            KTimer tu("kmeans_update", stream);
            hipLaunchKernelGGL(km_iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, sv0, n);
            if (hipMemcpyAsync(sk0, d_labels, 4 * nn, hipMemcpyDeviceToDevice, stream) != hipSuccess) {
                fail = true;
                break;
            }
            hipcub::DoubleBuffer<uint32_t> kb(sk0, sk1);
            hipcub::DoubleBuffer<int32_t> vb(sv0, sv1);
            size_t ts = tmp_sort;
            int end_bit = 1;
            while ((1 << end_bit) <= k) end_bit++;
            if (hipcub::DeviceRadixSort::SortPairs(tmp, ts, kb, vb, (int)n, 0, end_bit, stream) != hipSuccess) {
                fail = true;
                break;
            }
            hipLaunchKernelGGL(km_seg_kernel, dim3((k + 256) / 256), dim3(256), 0, stream, kb.Current(), n, k, d_seg);
            if (hipMemcpyAsync(seg.data(), d_seg, 4 * (size_t)(k + 1), hipMemcpyDeviceToHost, stream) != hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess) {
                fail = true;
                break;
            }
            rfirst.clear();
            rcount.clear();
            for (int c = 0; c < k; c++) {
                crun[c] = (int)rfirst.size();
                for (int b = seg[c]; b < seg[c + 1]; b += KM_RUN) {
                    rfirst.push_back(b);
                    rcount.push_back(std::min(KM_RUN, seg[c + 1] - b));
                }
            }
            crun[k] = (int)rfirst.size();
            const int R = crun[k];
            if (hipMemcpyAsync(d_rfirst, rfirst.data(), 4 * (size_t)R, hipMemcpyHostToDevice, stream) != hipSuccess ||
                hipMemcpyAsync(d_rcount, rcount.data(), 4 * (size_t)R, hipMemcpyHostToDevice, stream) != hipSuccess ||
                hipMemcpyAsync(d_crun, crun.data(), 4 * (size_t)(k + 1), hipMemcpyHostToDevice, stream) != hipSuccess) {
                fail = true;
                break;
            }
            if (R > 0)
                hipLaunchKernelGGL(km_partial_kernel, dim3(R), dim3(256), 0, stream, d_X, d, vb.Current(), d_rfirst,
                                   d_rcount, partial);
            hipLaunchKernelGGL(km_mean_kernel, dim3((unsigned)(((long)k * d + 255) / 256)), dim3(256), 0, stream,
                               partial, d, k, d_crun, d_seg, d_cent);
            if (hipGetLastError() != hipSuccess || hipStreamSynchronize(stream) != hipSuccess) {  // rfirst reuse
                fail = true;
                break;
            }
        }
        if (fail) break;
        rc = 0;
    } while (0);
    if (rc) set_error("kmeans: HIP failure");
    (void)hipStreamSynchronize(stream);
    (void)hipFree(ws);
    if (iterations) *iterations = it;
    return rc;
}

// PrepareDitherTiles (main.pas:2097-2152) for one keyframe: its tiles' LAB descriptors (UseWavelets as given,
// ADitheringGamma) -> k-means over them -> DitheringPalIndex = labels, PaletteCentroids = centroids.  Fewer than
// two tiles or palettes: every label 0, centroids 0 (main.pas:2135-2138 leaves PaletteCentroids zeroed).
int prepare_dither_dev(long n_tiles, const int32_t *d_rgb, int P, int gamma, int use_wavelets, int max_iter,
                       uint32_t seed, int32_t *d_labels, double *d_cent, int *iterations, hipStream_t stream) {
    if (n_tiles < 0 || P <= 0 || (n_tiles > 0 && (!d_rgb || !d_labels)) || !d_cent) {
        set_error("prepare_dither: invalid arguments");
        return -1;
    }
    if (iterations) *iterations = 0;
    if (n_tiles <= 1 || P <= 1) {
        if (n_tiles > 0) TILER_HIP_CHECK(hipMemsetAsync(d_labels, 0, 4 * (size_t)n_tiles, stream));
        TILER_HIP_CHECK(hipMemsetAsync(d_cent, 0, 8 * (size_t)P * 192, stream));
        TILER_HIP_CHECK(hipStreamSynchronize(stream));
        return 0;
    }
    double *X = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&X, 8 * (size_t)n_tiles * 192));
    PsyvArgs a;
    a.n = n_tiles;
    a.rgb = d_rgb;
    a.flags = PSYV_LAB | (use_wavelets ? PSYV_WAVELETS : 0);  // ComputeTilePsyVisFeatures(.., False, UseWavelets, True, ..)
    a.gamma = gamma;
    a.out64 = X;
    int rc = launch_psyv(a, stream);
    if (rc == 0) rc = kmeans_dev(X, n_tiles, 192, P, max_iter, seed, d_labels, d_cent, iterations, stream);
    (void)hipStreamSynchronize(stream);
    (void)hipFree(X);
    return rc;
}

}  // namespace tiler

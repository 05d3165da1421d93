// keyframes.hip -- the Load step's keyframe detection on gfx950:
//   ComputeInterFrameCorrelation main.pas:811-828 / PearsonCorrelation main.pas:1465-1492 over LoadFrame's
//   FSPixels (main.pas:3248-3262), and the shot-transition split of btnLoadClick main.pas:1099-1146.
//
// FSPixels are the r, g, b bytes of each screen pixel: with cBitsPerComp = 8 the Floyd-Steinberg pass over
// them (main.pas:1966-1993) posterizes with Posterize(v) = v (main.pas:703-709), so it changes nothing and the
// bytes are read straight from the frame tiles ([Q][64] int32 0x00BBGGRR, tile-major) in screen raster order.
//
// Bit-exact plan.  The reference's Pearson is ONE sequential fp64 pass (planar r, g, b; raster order), so the
// three sums are rounded in that exact order and cannot be re-associated.  What can be shared:
//   * mean(x) = Sum / N: the sum of bytes is an exact integer -> a parallel u64 reduction (frame_sum_kernel);
//   * Σ (x - m_f)^2 of frame f is the SAME rounded sequence whether f is the "x" of pair (f, f+1) or the "y"
//     of pair (f-1, f): it is computed once per frame (d2[f]);
//   * one LANE per frame runs the ordered chains d2[f] and num[f] = Σ (x_f - m_f)(x_{f+1} - m_{f+1}), the y term
//     coming from the neighbour lane; in the default form three producer waves compute the rounded terms into
//     LDS and one consumer wave only adds them in order (pearson_chain_pc_kernel).
// The chains are issue-bound fp64 work, not HBM-bound: a workgroup covers 60 frame pairs, so a launch costs about
// one frame's worth of sequential steps whatever F is.
// sqrt / product / division (4 flops per pair) finish on the host in double, as written in main.pas:1485-1491.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "keyframes.hpp"

namespace tiler {

// per frame: exact u64 sum of its r+g+b bytes (mean(x) main.pas:1472-1473)
__global__ __launch_bounds__(256) void frame_sum_kernel(const int4 *__restrict__ rgb, long vec_per_frame,
                                                          unsigned long long *__restrict__ sums) {
    const int f = blockIdx.y;
    const int4 *src = rgb + (long)f * vec_per_frame;
    unsigned long long acc = 0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < vec_per_frame; i += (long)gridDim.x * blockDim.x) {
        const int4 v = src[i];
        const unsigned w[4] = {(unsigned)v.x, (unsigned)v.y, (unsigned)v.z, (unsigned)v.w};
        unsigned s = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) s += (w[k] & 0xffu) + ((w[k] >> 8) & 0xffu) + ((w[k] >> 16) & 0xffu);
        acc += s;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(&sums[f], acc);
}

// One lane per frame (60 per wave, see below) runs, in the reference's order
// (channel-major, then screen raster: ya[i + sz*c] := FSPixels[i*3 + c], main.pas:819-826), the chains
// d2[f] = Σ (x_f - m_f)^2 and num[f] = Σ (x_f - m_f)(x_{f+1} - m_{f+1}); every op rounded (-ffp-contract=off).
// The y term of a pair is the NEXT lane's x term (same element, frame f+1), handed over by a DPP row shift
// (2 v_mov_dpp; a ds_bpermute shuffle cost 30 % of the kernel), so each lane streams one frame and each element
// costs one extract, one convert, one subtract, two moves, two multiplies and two adds (a per-lane LDS table of
// x - m instead of convert + subtract measured 8 % slower: 189 vs 175 ms for 1,000 1080p frames).  With one wave per SIMD
// nothing hides memory latency, so tile rows stream through a register ring KF_DEPTH rows ahead.
constexpr int KF_FRAMES_PER_WAVE = 60;

// lane i <- lane i+1 of the same 16-lane row (DPP row_shl:1); lane 15 of a row gets 0 (never used)
__device__ __forceinline__ double row_next(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x101, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x101, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int KF_DEPTH, int MODE>
__global__ __launch_bounds__(64) void pearson_chain_kernel(const int32_t *__restrict__ rgb, int F, int tm_w, int tm_h,
                                                           const unsigned long long *__restrict__ sums,
                                                           double *__restrict__ d2, double *__restrict__ num) {
    const int lane = threadIdx.x;
    // 4 rows of 16 lanes; in each row lanes 0..14 own frames and lane 15 feeds lane 14 (DPP row shifts stay
    // inside a row), so a wave owns 60 frames
    const int f = blockIdx.x * KF_FRAMES_PER_WAVE + 15 * (lane >> 4) + (lane & 15);
    const int fl = f < F ? f : F - 1;  // lanes past the end replay the last frame (all lanes stay active)
    const long fs = (long)tm_w * tm_h * 64;
    const double m = (double)sums[fl] / (3.0 * (double)fs);
    const int4 *a = reinterpret_cast<const int4 *>(rgb + fl * fs);
    const int rows = tm_h * 8;
    const long total = 3L * rows * tm_w;  // tile rows of 8 pixels, in summation order
    int lc = 0, lsy = 0, ltx = 0;         // load cursor (channel, screen row, tile column)
    int4 r0[KF_DEPTH], r1[KF_DEPTH];
    int sh[KF_DEPTH];
    auto load_next = [&](int4 &v0, int4 &v1, int &s) {
        const long o = (((long)(lsy >> 3) * tm_w + ltx) * 64 + (lsy & 7) * 8) >> 2;
        v0 = a[o];
        v1 = a[o + 1];
        s = 8 * lc;
        if (++ltx == tm_w) {
            ltx = 0;
            if (++lsy == rows) {
                lsy = 0;
                lc = lc == 2 ? 0 : lc + 1;  // past the end: harmless re-reads, never summed
            }
        }
    };
#pragma unroll
    for (int d = 0; d < KF_DEPTH; d++) load_next(r0[d], r1[d], sh[d]);
    double acc_n = 0.0, acc_d = 0.0, acc_n2 = 0.0, acc_d2 = 0.0;
    for (long j = 0; j < total; j += KF_DEPTH) {
#pragma unroll
        for (int d = 0; d < KF_DEPTH; d++) {
            const int4 v0 = r0[d], v1 = r1[d];
            const int s = sh[d];
            load_next(r0[d], r1[d], sh[d]);
            if (j + d < total) {
                const int w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
                double dx[8], dy[8];
#pragma unroll
                for (int k = 0; k < 8; k++) dx[k] = (double)__builtin_amdgcn_ubfe((unsigned)w[k], (unsigned)s, 8u) - m;
#pragma unroll
                for (int k = 0; k < 8; k++) dy[k] = MODE == 1 ? dx[k] : row_next(dx[k]);
                if (MODE == 2) {  // timing experiment only (re-associated, NOT the reference's result)
#pragma unroll
                    for (int k = 0; k < 8; k += 2) {
                        acc_n = acc_n + dx[k] * dy[k];
                        acc_d = acc_d + dx[k] * dx[k];
                        acc_n2 = acc_n2 + dx[k + 1] * dy[k + 1];
                        acc_d2 = acc_d2 + dx[k + 1] * dx[k + 1];
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        acc_n = acc_n + dx[k] * dy[k];
                        acc_d = acc_d + dx[k] * dx[k];
                    }
                }
            }
        }
    }
    if (MODE == 2) {
        acc_n = acc_n + acc_n2;
        acc_d = acc_d + acc_d2;
    }
    if ((lane & 15) < 15 && f < F) {
        d2[f] = acc_d;
        if (f + 1 < F) num[f] = acc_n;
    }
}

// Producer/consumer form (default).  The chain adds are the only sequential part; everything else per element
// (extract, convert, subtract, neighbour move, two multiplies) is independent across elements.  A workgroup of
// 4 waves serves the same 60 frames: waves 1-3 compute the rounded products (x-m_f)(x'-m_{f+1}) and (x-m_f)^2
// of a stage of KF_STAGE elements into LDS, wave 0 only adds them in sequence order (one LDS read + two adds per
// element), double-buffered with one barrier per stage.  Same terms, same order: bit-identical to the lane form.
// Measured (1,000 random 1080p frames, one MI355X): lane form 175 ms; this form with 60 frames per workgroup
// 122 ms (consumer idle: 130 ms, producers idle: 70 ms; 4 producers or a 4-stage fetch ring: no change), with
// 30 frames 89 ms, with 15 frames 84 ms (default: 15 frames = one DPP row per workgroup, the other rows mirror
// it) -- the 60 scattered frame streams of one CU were limited by that CU's outstanding misses; 70 ms is the
// consumer's floor (one LDS read and two chained fp64 adds per element).
template <int MODE, int KF_PRODUCERS, int KF_ROWS_PER_PRODUCER, int KF_PD, int KF_DPP_ROWS>
__global__ __launch_bounds__(512) void pearson_chain_pc_kernel(const int32_t *__restrict__ rgb, int F, int tm_w,
                                                               int tm_h, const unsigned long long *__restrict__ sums,
                                                               double *__restrict__ d2, double *__restrict__ num) {
    constexpr int KF_STAGE_ROWS = KF_PRODUCERS * KF_ROWS_PER_PRODUCER;  // tile rows (8 elements) per stage
    constexpr int KF_STAGE = KF_STAGE_ROWS * 8;
    static_assert(2 * KF_STAGE * 64 * 16 <= 160 * 1024, "stage ring exceeds the LDS");
    __shared__ double2 s_t[2][KF_STAGE][64];  // (num term, d2 term) per element and lane
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // KF_DPP_ROWS of the 4 DPP rows own frames (15 each); the other rows mirror them (same addresses, so their
    // loads merge): fewer frames per CU, more CUs streaming
    const int f = blockIdx.x * 15 * KF_DPP_ROWS + 15 * ((lane >> 4) % KF_DPP_ROWS) + (lane & 15);
    const int fl = f < F ? f : F - 1;
    const long fs = (long)tm_w * tm_h * 64;
    const int rows = tm_h * 8;
    const long total = 3L * rows * tm_w;  // tile rows in summation order
    const long nstage = (total + KF_STAGE_ROWS - 1) / KF_STAGE_ROWS;
    if (w > 0) {
        // ---- producer p = w-1: tile rows 9s + 3p + {0,1,2} of stage s ----
        const int p = w - 1;
        const double m = (double)sums[fl] / (3.0 * (double)fs);
        const int4 *a = reinterpret_cast<const int4 *>(rgb + fl * fs);
        // tile-row cursor (channel, screen row, tile column) of this producer's first row of the next stage to
        // fetch; it advances by KF_STAGE_ROWS per stage (no divisions in the loop)
        int cc = 0, csy = 0, ctx = 0;
        auto advance = [&](int n) {
            ctx += n;
            while (ctx >= tm_w) {
                ctx -= tm_w;
                if (++csy == rows) {
                    csy = 0;
                    ++cc;
                }
            }
        };
        advance(p * KF_ROWS_PER_PRODUCER);
        // register ring: stage s lives in slot s % KF_PD, fetched KF_PD stages ahead (one wave per producer
        // slot has little else to hide a global-load latency with)
        int4 n0[KF_PD][KF_ROWS_PER_PRODUCER], n1[KF_PD][KF_ROWS_PER_PRODUCER];
        int ns[KF_PD][KF_ROWS_PER_PRODUCER];
        auto fetch = [&](int4 *v0, int4 *v1, int *vs) {  // rows beyond the end re-read the last row (never summed)
            int c = cc, sy = csy, tx = ctx;
#pragma unroll
            for (int i = 0; i < KF_ROWS_PER_PRODUCER; i++) {
                if (c > 2) {
                    c = 2;
                    sy = rows - 1;
                    tx = tm_w - 1;
                }
                const long o = (((long)(sy >> 3) * tm_w + tx) * 64 + (sy & 7) * 8) >> 2;
                v0[i] = a[o];
                v1[i] = a[o + 1];
                vs[i] = 8 * c;
                if (++tx == tm_w) {
                    tx = 0;
                    if (++sy == rows) {
                        sy = 0;
                        ++c;
                    }
                }
            }
            advance(KF_STAGE_ROWS);
        };
#pragma unroll
        for (int q = 0; q < KF_PD; q++) fetch(n0[q], n1[q], ns[q]);
        for (long s0 = 0; s0 < nstage; s0 += KF_PD) {
#pragma unroll
            for (int q = 0; q < KF_PD; q++) {
                const long st = s0 + q;
                if (st < nstage) {
                    int4 c0[KF_ROWS_PER_PRODUCER], c1[KF_ROWS_PER_PRODUCER];
                    int cs[KF_ROWS_PER_PRODUCER];
#pragma unroll
                    for (int i = 0; i < KF_ROWS_PER_PRODUCER; i++) {
                        c0[i] = n0[q][i];
                        c1[i] = n1[q][i];
                        cs[i] = ns[q][i];
                    }
                    if (st + KF_PD < nstage) fetch(n0[q], n1[q], ns[q]);
                    if (MODE != 5) {  // MODE 5: timing experiment, producers idle (results invalid)
                        double2 *buf = &s_t[st & 1][0][0];
#pragma unroll
                        for (int i = 0; i < KF_ROWS_PER_PRODUCER; i++) {
                            const int wv[8] = {c0[i].x, c0[i].y, c0[i].z, c0[i].w, c1[i].x, c1[i].y, c1[i].z, c1[i].w};
#pragma unroll
                            for (int e = 0; e < 8; e++) {
                                // (double)x exactly, without v_cvt_f64_u32: 2^52 + x built from its bits, minus 2^52
                                const double xb = __hiloint2double(
                                    0x43300000, (int)__builtin_amdgcn_ubfe((unsigned)wv[e], (unsigned)cs[i], 8u));
                                const double dx = (xb - 4503599627370496.0) - m;
                                const double dy = row_next(dx);
                                buf[((p * KF_ROWS_PER_PRODUCER + i) * 8 + e) * 64 + lane] =
                                    make_double2(dx * dy, dx * dx);
                            }
                        }
                    }
                    __syncthreads();
                }
            }
        }
        __syncthreads();
    } else {
        // ---- consumer: the two ordered chains ----
        double acc_n = 0.0, acc_d = 0.0;
        __syncthreads();
        for (long st = 0; st < nstage; st++) {
            const double2 *buf = &s_t[st & 1][0][0];
            const long left = (total - st * KF_STAGE_ROWS) * 8;
            if (MODE == 4) {  // timing experiment: consumer idle (results invalid)
            } else if (left >= KF_STAGE) {
#pragma unroll 8
                for (int e = 0; e < KF_STAGE; e++) {
                    const double2 t = buf[e * 64 + lane];
                    acc_n = acc_n + t.x;
                    acc_d = acc_d + t.y;
                }
            } else {
                for (int e = 0; e < (int)left; e++) {
                    const double2 t = buf[e * 64 + lane];
                    acc_n = acc_n + t.x;
                    acc_d = acc_d + t.y;
                }
            }
            __syncthreads();
        }
        if ((lane & 15) < 15 && (lane >> 4) < KF_DPP_ROWS && f < F) {
            d2[f] = acc_d;
            if (f + 1 < F) num[f] = acc_n;
        }
    }
}

int interframe_corr_dev(const int32_t *d_rgb, int F, int tm_w, int tm_h, double *corr, hipStream_t stream) {
    if (F < 0 || tm_w <= 0 || tm_h <= 0 || (F > 0 && !d_rgb) || (F > 1 && !corr)) {
        set_error("keyframes: invalid arguments");
        return -1;
    }
    if (F <= 1) return 0;
    if ((long)tm_w * tm_h > (1L << 24) || (uintptr_t)d_rgb % 16) {
        set_error("keyframes: frame too large or frames not 16-byte aligned");
        return -1;
    }
    const long fs = (long)tm_w * tm_h * 64;
    char *buf = nullptr;
    const size_t bytes = (size_t)F * 24;
    TILER_HIP_CHECK(hipMallocAsync((void **)&buf, bytes, stream));
    unsigned long long *d_sums = (unsigned long long *)buf;
    double *d_d2 = (double *)(buf + (size_t)F * 8), *d_num = (double *)(buf + (size_t)F * 16);
    std::vector<double> h(2 * (size_t)F);
    int rc = -1;
    do {
        if (hipMemsetAsync(d_sums, 0, (size_t)F * 8, stream) != hipSuccess) break;
        {
            KTimer tm("kf_sum", stream);
            const int bx = (int)std::min<long>(64, (fs / 4 + 4095) / 4096);
            hipLaunchKernelGGL(frame_sum_kernel, dim3(bx, F), dim3(256), 0, stream, (const int4 *)d_rgb, fs / 4,
                               d_sums);
            if (hipGetLastError() != hipSuccess) break;
        }
        {
            KTimer tm("kf_corr", stream);
            {
                const int per = 15;  // frames per workgroup (one DPP row; see the kernel)
                hipLaunchKernelGGL((pearson_chain_pc_kernel<0, 3, 3, 2, 1>), dim3((F + per - 1) / per), dim3(256), 0,
                                   stream, d_rgb, F, tm_w, tm_h, d_sums, d_d2, d_num);
            }
            if (hipGetLastError() != hipSuccess) break;
        }
        if (hipMemcpyAsync(h.data(), d_d2, (size_t)F * 16, hipMemcpyDeviceToHost, stream) != hipSuccess) break;
        if (hipStreamSynchronize(stream) != hipSuccess) break;
        rc = 0;
    } while (0);
    (void)hipFreeAsync(buf, stream);
    if (rc) {
        set_error(std::string("keyframes: HIP failure: ") + hipGetErrorString(hipGetLastError()));
        return -1;
    }
    // PearsonCorrelation tail main.pas:1485-1491
    for (int p = 0; p + 1 < F; p++) {
        const double denx = sqrt(h[p]), deny = sqrt(h[p + 1]);
        const double den = denx * deny;
        corr[p] = den != 0.0 ? h[F + p] / den : 0.0;
    }
    return 0;
}

int interframe_corr_host(const int32_t *rgb, int F, int tm_w, int tm_h, double *corr) {
    if (F < 0 || tm_w <= 0 || tm_h <= 0 || (F > 0 && !rgb) || (F > 1 && !corr)) {
        set_error("keyframes: invalid arguments");
        return -1;
    }
    if (F <= 1) return 0;
    const size_t bytes = (size_t)F * tm_w * tm_h * 64 * 4;
    int32_t *d = nullptr;
    hipStream_t st = nullptr;
    TILER_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int rc = -1;
    if (hipMalloc((void **)&d, bytes) == hipSuccess) {
        if (hipMemcpyAsync(d, rgb, bytes, hipMemcpyHostToDevice, st) == hipSuccess)
            rc = interframe_corr_dev(d, F, tm_w, tm_h, corr, st);
        else
            set_error("keyframes: host-to-device copy failed");
        (void)hipStreamSynchronize(st);
        (void)hipFree(d);
    } else {
        set_error("keyframes: device allocation failed");
    }
    (void)hipStreamDestroy(st);
    return rc;
}

// btnLoadClick main.pas:1099-1146: the shot-transition split over the correlations (host bookkeeping).
int find_keyframes(const double *corr, int F, int tile_map_size, int32_t *kf_of_frame) {
    if (F < 0 || tile_map_size < 0 || (F > 0 && !kf_of_frame) || (F > 1 && !corr)) {
        set_error("keyframes: invalid arguments");
        return -1;
    }
    if (F == 0) return 0;
    const long max_tiles_per_kf = 24L * 1920 * 1080 / 64;  // CShotTransMaxTilesPerKF (main.pas:986)
    const int grace = 24;                                  // CShotTransGracePeriod
    const double savg = 6;                                 // CShotTransSAvgFrames
    const double soft = 0.9, hard = 0.5;                   // CShotTransSoftThres / HardThres
    int kf = 0, last = 0;
    double av = -1.0;
    kf_of_frame[0] = 0;
    for (int i = 1; i < F; i++) {
        const double v = corr[i - 1];
        av = av == -1.0 ? v : av * (1.0 - 1.0 / savg) + v * (1.0 / savg);
        const double ratio = (0.01 > v ? 0.01 : v) / (0.01 > av ? 0.01 : av);  // Math.Max: if a > b then a else b
        const bool span = (long)(i - last + 1) * tile_map_size > max_tiles_per_kf;
        if (ratio < hard || (ratio < soft && (i - last + 1) > grace) || span) {
            kf++;
            av = -1.0;
            last = i;
        }
        kf_of_frame[i] = kf;
    }
    return kf + 1;
}

}  // namespace tiler

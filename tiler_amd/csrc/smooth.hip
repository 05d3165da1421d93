// smooth.hip -- Smooth step (btnSmoothClick main.pas:1338-1370 / DoTemporalSmoothing main.pas:4071-4119).
//
// Parallel over tilemap positions (one wave64 per position), sequential over the keyframe's frames,
// exactly the reference's dependency structure (rows in parallel, frames in order).  Per step:
//   descriptor of the current smoothed item: DCT branch, Q-weighting, gamma -1, item's own mirrors
//   (main.pas:4097-4098), fp64 in source order -> identical bits to the CPU restatement;
//   cmp = sqrt(sum_k (cur_k - prev_k)^2 * (1/192)) summed in index order (CompareEuclideanDCTPtr 659-675);
//   |cmp| <= Strength -> copy the lower-index item across (4102-4113).
// The previous item's descriptor is carried in registers (after a merge both sides hold the same item),
// so each step costs one descriptor: 3 x 64 x 64 fp64 MACs.
#include <math.h>

#include <algorithm>
#include <string>

#include "psyv_dev.hpp"
#include "smooth.hpp"

#pragma clang fp contract(off)

namespace tiler {

struct SmoothArgs {
    int F, Q;
    int32_t *tile, *tmpidx, *pal;
    uint8_t *hm, *vm, *sm;
    const uint8_t *palpix;
    const int32_t *palettes;
    double strength;
    PsyvConst k;
};

__device__ __forceinline__ void item_dct(const SmoothArgs &a, int tile, int pal, int hm, int vm, int lane,
                                         double (&out)[3]) {
    const int y = lane >> 3, x = lane & 7;
    const int xx = hm ? 7 - x : x, yy = vm ? 7 - y : y;
    const int32_t col = a.palettes[(long)pal * 16 + a.palpix[(long)tile * 64 + yy * 8 + xx]];
    double cp[3];
    yuv_of(col, a.k.gamma_lut, a.k.u_mul, a.k.v_mul, cp[0], cp[1], cp[2]);  // gamma -1: LUT row 0 = i/255
#pragma unroll
    for (int c = 0; c < 3; c++) out[c] = dct_lane(cp[c], lane, c, true, a.k);
}

__global__ __launch_bounds__(256) void smooth_kernel(SmoothArgs a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double inv = 1.0 / (64.0 * 3.0);  // cSqrtFactor main.pas:4073
    for (long s = (long)blockIdx.x * 4 + wave; s < a.Q; s += (long)gridDim.x * 4) {
        int pt = a.tile[s], pp = a.pal[s], ph = a.hm[s], pv = a.vm[s], ps = a.sm[s];
        int ptmp = a.tmpidx ? a.tmpidx[s] : 0;
        double pd[3];
        item_dct(a, pt, pp, ph, pv, lane, pd);
        for (int i = 1; i < a.F; i++) {
            const long c = (long)i * a.Q + s, p = (long)(i - 1) * a.Q + s;
            const int ct = a.tile[c], cpl = a.pal[c], chm = a.hm[c], cvm = a.vm[c], csm = a.sm[c];
            const int ctmp = a.tmpidx ? a.tmpidx[c] : 0;
            double cd[3];
            item_dct(a, ct, cpl, chm, cvm, lane, cd);
            double sq[3];
#pragma unroll
            for (int cc = 0; cc < 3; cc++) {
                const double t = cd[cc] - pd[cc];
                sq[cc] = t * t;
            }
            // sequential sum over k = 0..191 (every lane accumulates the same sequence: uniform result)
            double acc = 0.0;
#pragma unroll
            for (int cc = 0; cc < 3; cc++)
                for (int j = 0; j < 64; j++) acc += shfl_d(sq[cc], j);
            const double cmp = sqrt(acc * inv);
            const bool smooth = fabs(cmp) <= a.strength;
            if (smooth) {
                if (ct >= pt) {  // TMI^ := PrevTMI^ ; TMI^.Smoothed := True
                    if (lane == 0) {
                        a.tile[c] = pt;
                        a.pal[c] = pp;
                        a.hm[c] = (uint8_t)ph;
                        a.vm[c] = (uint8_t)pv;
                        a.sm[c] = 1;
                        if (a.tmpidx) a.tmpidx[c] = ptmp;
                    }
                    ps = 1;  // prev item unchanged, descriptor unchanged
                } else {         // PrevTMI^ := TMI^ ; TMI^.Smoothed := True
                    if (lane == 0) {
                        a.tile[p] = ct;
                        a.pal[p] = cpl;
                        a.hm[p] = (uint8_t)chm;
                        a.vm[p] = (uint8_t)cvm;
                        a.sm[p] = (uint8_t)csm;
                        if (a.tmpidx) a.tmpidx[p] = ctmp;
                        a.sm[c] = 1;
                    }
                    pt = ct, pp = cpl, ph = chm, pv = cvm, ps = 1, ptmp = ctmp;
#pragma unroll
                    for (int cc = 0; cc < 3; cc++) pd[cc] = cd[cc];
                }
            } else {
                if (lane == 0) a.sm[c] = 0;
                pt = ct, pp = cpl, ph = chm, pv = cvm, ps = 0, ptmp = ctmp;
#pragma unroll
                for (int cc = 0; cc < 3; cc++) pd[cc] = cd[cc];
            }
        }
        (void)ps;
    }
}

int smooth_keyframe_dev(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                        uint8_t *sm, const uint8_t *palpix, const int32_t *palettes, double strength,
                        hipStream_t stream) {
    if (F <= 1 || Q <= 0) return 0;
    const Luts &L = luts();
    SmoothArgs a{F, Q, tile, tmpidx, pal, hm, vm, sm, palpix, palettes, strength,
                 PsyvConst{L.d_gamma, L.d_dct, L.d_qmul, L.d_ratio, L.haar_f, L.u_mul, L.v_mul}};
    const long blocks = std::min<long>(65536, (Q + 3) / 4);
    KTimer tm("smooth", stream);
    hipLaunchKernelGGL(smooth_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

int smooth_keyframe_host(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                         uint8_t *smoothed, int T, const uint8_t *palpix, int P, const int32_t *palettes,
                         double strength) {
    if (F < 0 || Q < 0 || T < 0 || P < 0 || (F * (long)Q > 0 && (!tile || !pal || !hm || !vm || !smoothed))) {
        set_error("smooth: invalid arguments");
        return -1;
    }
    if (F <= 1 || Q == 0) return 0;
    if (!palpix || !palettes || T <= 0 || P <= 0) {
        set_error("smooth: tiles / palettes missing");
        return -1;
    }
    const long n = (long)F * Q;
    for (long i = 0; i < n; i++)
        if (tile[i] < 0 || tile[i] >= T || pal[i] < 0 || pal[i] >= P) {
            set_error("smooth: tile or palette index out of range");
            return -1;
        }
    char *buf = nullptr;
    const size_t sz_i = n * 4, sz_b = n;
    const size_t total = 3 * sz_i + 3 * sz_b + (size_t)T * 64 + (size_t)P * 64 + 64;
    TILER_HIP_CHECK(hipMalloc((void **)&buf, total));
    int32_t *d_tile = (int32_t *)buf, *d_tmp = d_tile + n, *d_pal = d_tmp + n;
    uint8_t *d_hm = (uint8_t *)(d_pal + n), *d_vm = d_hm + n, *d_sm = d_vm + n;
    uint8_t *d_pp = d_sm + n;
    int32_t *d_pals = (int32_t *)(((uintptr_t)(d_pp + (size_t)T * 64) + 15) & ~(uintptr_t)15);
    hipStream_t st = nullptr;
    int rc = -1;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        hipFree(buf);
        set_error("smooth: stream creation failed");
        return -1;
    }
    do {
        if (hipMemcpyAsync(d_tile, tile, sz_i, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (tmpidx && hipMemcpyAsync(d_tmp, tmpidx, sz_i, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_pal, pal, sz_i, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_hm, hm, sz_b, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_vm, vm, sz_b, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_sm, smoothed, sz_b, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_pp, palpix, (size_t)T * 64, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_pals, palettes, (size_t)P * 64, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (smooth_keyframe_dev(F, Q, d_tile, tmpidx ? d_tmp : nullptr, d_pal, d_hm, d_vm, d_sm, d_pp, d_pals, strength,
                                st))
            break;
        if (hipMemcpyAsync(tile, d_tile, sz_i, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (tmpidx && hipMemcpyAsync(tmpidx, d_tmp, sz_i, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(pal, d_pal, sz_i, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(hm, d_hm, sz_b, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(vm, d_vm, sz_b, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(smoothed, d_sm, sz_b, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        rc = 0;
    } while (0);
    if (rc) set_error(std::string("smooth: HIP failure: ") + last_error());
    (void)hipStreamDestroy(st);
    (void)hipFree(buf);
    return rc;
}

}  // namespace tiler

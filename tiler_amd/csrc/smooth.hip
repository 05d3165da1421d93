// smooth.hip -- Smooth step (btnSmoothClick main.pas:1338-1370 / DoTemporalSmoothing main.pas:4071-4119).
//
// Parallel over tilemap positions, sequential over the keyframe's frames -- exactly the reference's
// dependency structure (rows in parallel, frames in order).  Per step the reference computes two DCT
// descriptors (DCT branch, Q-weighting, gamma -1, the item's own mirrors, main.pas:4097-4098) and
//   cmp = sqrt(sum_k (cur_k - prev_k)^2 * (1/192)) summed in index order (CompareEuclideanDCTPtr 659-675);
//   |cmp| <= Strength -> copy the lower-index item across (4102-4113).
// A descriptor is a pure function of (tile, palette, H, V), and a keyframe's tilemaps reuse few distinct
// items, so each distinct item's descriptor is computed ONCE (bit-identical: psyv_kernel, fp64 in source
// order) into a per-call table, and the chain kernel (one thread per position) only streams two table rows
// per step through the sequential fp64 sum.  Distinct items are found with a GPU hash in three passes
// (insert keys / number the slots / look items up: no spinning on another lane's write).
#include <math.h>

#include <algorithm>
#include <string>

#include "psyv.hpp"
#include "psyv_dev.hpp"
#include "smooth.hpp"

#pragma clang fp contract(off)

namespace tiler {

static constexpr unsigned long long SM_EMPTY = ~0ull;

__device__ __forceinline__ unsigned long long sm_key(int tile, int pal, int hm, int vm) {
    return ((unsigned long long)(unsigned)tile << 32) | ((unsigned long long)((unsigned)pal & 0x3FFFFFFFu) << 2) |
           (hm ? 2ull : 0ull) | (vm ? 1ull : 0ull);
}
__device__ __forceinline__ unsigned sm_hash(unsigned long long k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (unsigned)k;
}

struct SmoothHash {
    unsigned long long *keys;  // [cap]
    int32_t *vals;             // [cap]
    unsigned mask;
    int32_t *count;            // [1]
    int32_t *u_tile, *u_pal;   // [n] distinct items
    uint8_t *u_flags;          // psyv mirror flags of each distinct item
    int32_t *didx;             // [n] descriptor row of every item
};

__global__ __launch_bounds__(256) void smooth_hash_insert(long n, const int32_t *tile, const int32_t *pal,
                                                          const uint8_t *hm, const uint8_t *vm, SmoothHash h) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const unsigned long long k = sm_key(tile[i], pal[i], hm[i], vm[i]);
        unsigned p = sm_hash(k) & h.mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&h.keys[p], SM_EMPTY, k);
            if (prev == SM_EMPTY || prev == k) break;
            p = (p + 1) & h.mask;
        }
    }
}

__global__ __launch_bounds__(256) void smooth_hash_number(SmoothHash h, long cap) {
    for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < cap; p += (long)gridDim.x * 256) {
        const unsigned long long k = h.keys[p];
        if (k == SM_EMPTY) continue;
        const int idx = atomicAdd(h.count, 1);
        h.vals[p] = idx;
        h.u_tile[idx] = (int)(k >> 32);
        h.u_pal[idx] = (int)((k >> 2) & 0x3FFFFFFFu);
        h.u_flags[idx] = (uint8_t)(((k & 2) ? PSYV_HMIRROR : 0) | ((k & 1) ? PSYV_VMIRROR : 0));
    }
}

__global__ __launch_bounds__(256) void smooth_hash_lookup(long n, const int32_t *tile, const int32_t *pal,
                                                          const uint8_t *hm, const uint8_t *vm, SmoothHash h) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const unsigned long long k = sm_key(tile[i], pal[i], hm[i], vm[i]);
        unsigned p = sm_hash(k) & h.mask;
        while (h.keys[p] != k) p = (p + 1) & h.mask;
        h.didx[i] = h.vals[p];
    }
}

struct SmoothArgs {
    int F, Q;
    int32_t *tile, *tmpidx, *pal;
    uint8_t *hm, *vm, *sm;
    const int32_t *didx;   // [F][Q] descriptor row of every item
    const double *desc;    // [U][192]
    double strength;
};

// sum_{k < 192} (a_k - b_k)^2 in index order, fp64, every op rounded (CompareEuclideanDCTPtr 659-675)
__device__ __forceinline__ double sq_dist192(const double *__restrict__ a, const double *__restrict__ b) {
    const double2 *a2 = reinterpret_cast<const double2 *>(a), *b2 = reinterpret_cast<const double2 *>(b);
    double acc = 0.0;
#pragma unroll 8
    for (int k = 0; k < 96; k++) {
        const double2 x = a2[k], y = b2[k];
        double t = x.x - y.x;
        acc += t * t;
        t = x.y - y.y;
        acc += t * t;
    }
    return acc;
}

__global__ __launch_bounds__(64) void smooth_chain_kernel(SmoothArgs a) {
    const double inv = 1.0 / (64.0 * 3.0);  // cSqrtFactor main.pas:4073
    for (long s = (long)blockIdx.x * 64 + threadIdx.x; s < a.Q; s += (long)gridDim.x * 64) {
        int pt = a.tile[s], pp = a.pal[s], ph = a.hm[s], pv = a.vm[s];
        int ptmp = a.tmpidx ? a.tmpidx[s] : 0;
        int pdi = a.didx[s];
        for (int i = 1; i < a.F; i++) {
            const long c = (long)i * a.Q + s, p = (long)(i - 1) * a.Q + s;
            const int ct = a.tile[c], cpl = a.pal[c], chm = a.hm[c], cvm = a.vm[c], csm = a.sm[c];
            const int ctmp = a.tmpidx ? a.tmpidx[c] : 0;
            const int cdi = a.didx[c];
            const double acc = sq_dist192(a.desc + (long)cdi * 192, a.desc + (long)pdi * 192);  // cur - prev
            const double cmp = sqrt(acc * inv);
            if (fabs(cmp) <= a.strength) {
                if (ct >= pt) {  // TMI^ := PrevTMI^ ; TMI^.Smoothed := True (prev item and descriptor unchanged)
                    a.tile[c] = pt;
                    a.pal[c] = pp;
                    a.hm[c] = (uint8_t)ph;
                    a.vm[c] = (uint8_t)pv;
                    a.sm[c] = 1;
                    if (a.tmpidx) a.tmpidx[c] = ptmp;
                } else {  // PrevTMI^ := TMI^ ; TMI^.Smoothed := True
                    a.tile[p] = ct;
                    a.pal[p] = cpl;
                    a.hm[p] = (uint8_t)chm;
                    a.vm[p] = (uint8_t)cvm;
                    a.sm[p] = (uint8_t)csm;
                    if (a.tmpidx) a.tmpidx[p] = ctmp;
                    a.sm[c] = 1;
                    pt = ct, pp = cpl, ph = chm, pv = cvm, ptmp = ctmp, pdi = cdi;
                }
            } else {
                a.sm[c] = 0;
                pt = ct, pp = cpl, ph = chm, pv = cvm, ptmp = ctmp, pdi = cdi;
            }
        }
    }
}

int smooth_keyframe_dev(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                        uint8_t *sm, const uint8_t *palpix, const int32_t *palettes, double strength,
                        hipStream_t stream) {
    if (F <= 1 || Q <= 0) return 0;
    const long n = (long)F * Q;
    long cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    // scratch (stream-ordered): hash keys/vals, distinct items, item -> row
    char *buf = nullptr;
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_keys = carve(cap * 8), o_vals = carve(cap * 4), o_cnt = carve(4), o_ut = carve(n * 4),
                 o_up = carve(n * 4), o_uf = carve(n), o_didx = carve(n * 4);
    KTimer tm("smooth", stream);
    TILER_HIP_CHECK(hipMallocAsync((void **)&buf, off, stream));
    SmoothHash h{(unsigned long long *)(buf + o_keys), (int32_t *)(buf + o_vals), (unsigned)(cap - 1),
                 (int32_t *)(buf + o_cnt), (int32_t *)(buf + o_ut), (int32_t *)(buf + o_up), (uint8_t *)(buf + o_uf),
                 (int32_t *)(buf + o_didx)};
    int rc = -1;
    double *desc = nullptr;
    do {
        if (hipMemsetAsync(h.keys, 0xff, cap * 8, stream) != hipSuccess) break;
        if (hipMemsetAsync(h.count, 0, 4, stream) != hipSuccess) break;
        const unsigned g = (unsigned)std::min<long>(8192, (n + 255) / 256);
        hipLaunchKernelGGL(smooth_hash_insert, dim3(g), dim3(256), 0, stream, n, tile, pal, hm, vm, h);
        hipLaunchKernelGGL(smooth_hash_number, dim3((unsigned)std::min<long>(8192, (cap + 255) / 256)), dim3(256), 0,
                           stream, h, cap);
        hipLaunchKernelGGL(smooth_hash_lookup, dim3(g), dim3(256), 0, stream, n, tile, pal, hm, vm, h);
        int U = 0;
        if (hipMemcpyAsync(&U, h.count, 4, hipMemcpyDeviceToHost, stream) != hipSuccess) break;
        if (hipStreamSynchronize(stream) != hipSuccess) break;
        if (hipMallocAsync((void **)&desc, (size_t)std::max(U, 1) * 192 * 8, stream) != hipSuccess) break;
        // the distinct items' descriptors, exactly as item by item (DCT, Q-weighting, gamma -1, own mirrors)
        PsyvArgs pa;
        pa.n = U;
        pa.palpix = palpix;
        pa.tile_of = h.u_tile;
        pa.palettes = palettes;
        pa.pal_of = h.u_pal;
        pa.flags_per = h.u_flags;
        pa.flags = PSYV_FROM_PAL | PSYV_QWEIGHT;
        pa.gamma = -1;
        pa.out64 = desc;
        if (launch_psyv(pa, stream)) break;
        SmoothArgs a{F, Q, tile, tmpidx, pal, hm, vm, sm, h.didx, desc, strength};
        // one thread per position, one wave per block: the few waves of a keyframe spread over every CU
        hipLaunchKernelGGL(smooth_chain_kernel, dim3((unsigned)std::max<long>(1, std::min<long>(65536, (Q + 63) / 64))),
                           dim3(64), 0, stream, a);
        if (hipGetLastError() != hipSuccess) break;
        rc = 0;
    } while (0);
    if (desc) (void)hipFreeAsync(desc, stream);
    (void)hipFreeAsync(buf, stream);
    if (rc) {
        set_error(std::string("smooth: HIP failure: ") + hipGetErrorString(hipGetLastError()));
        return -1;
    }
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

// smooth.hip -- Smooth step (btnSmoothClick main.pas:1338-1370 / DoTemporalSmoothing main.pas:4071-4119).
//
// Parallel over tilemap positions, sequential over the keyframe's frames -- exactly the reference's
// dependency structure (rows in parallel, frames in order).  Per step the reference computes two DCT
// descriptors (DCT branch, Q-weighting, gamma -1, the item's own mirrors, main.pas:4097-4098) and
//   cmp = sqrt(sum_k (cur_k - prev_k)^2 * (1/192)) summed in index order (CompareEuclideanDCTPtr 659-675);
//   |cmp| <= Strength -> copy the lower-index item across (4102-4113).
// A descriptor is a pure function of (tile, palette, H, V), and a keyframe's tilemaps reuse few distinct
// items, so each distinct item's descriptor is computed ONCE (bit-identical: psyv_kernel, fp64 in source
// order) into a per-call table, and the chain kernel (8 lanes per position) reads one table row per step
// (the previous item's row stays in registers) into the sequential fp64 sum.  Distinct items are found with a GPU hash in three passes
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

// A keyframe's tilemaps repeat items heavily (flat regions, static positions), and many lanes inserting the same key
// at once serialise on one slot's atomics (0.33 ms at C3).  Only the first lane of each distinct key in a wave
// inserts (pairwise compare over the wave), and a plain read settles keys already present.
__global__ __launch_bounds__(256) void smooth_hash_insert(long n, const int32_t *tile, const int32_t *pal,
                                                          const uint8_t *hm, const uint8_t *vm, SmoothHash h) {
    const int lane = threadIdx.x & 63;
    const long n_up = (n + 63) & ~63L;  // uniform trip count per wave (the shuffles need every lane)
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n_up; i += (long)gridDim.x * 256) {
        const bool act = i < n;
        const unsigned long long k = act ? sm_key(tile[i], pal[i], hm[i], vm[i]) : SM_EMPTY;
        const unsigned klo = (unsigned)k, khi = (unsigned)(k >> 32);
        bool dup = !act;
        for (int d = 1; d < 64; d++) {
            const int src = (lane - d) & 63;
            const unsigned olo = __shfl(klo, src, 64), ohi = __shfl(khi, src, 64);
            dup |= lane >= d && olo == klo && ohi == khi;
        }
        if (dup) continue;
        unsigned p = sm_hash(k) & h.mask;
        for (;;) {
            // most items repeat across the keyframe's frames: a plain read settles a slot that already holds
            // the key without an L2 atomic (a stale read only falls through to the CAS, which decides)
            const unsigned long long seen = __builtin_nontemporal_load(&h.keys[p]);
            if (seen == k) break;
            if (seen == SM_EMPTY) {
                const unsigned long long prev = atomicCAS(&h.keys[p], SM_EMPTY, k);
                if (prev == SM_EMPTY || prev == k) break;
            }
            p = (p + 1) & h.mask;
        }
    }
}

// Numbers the occupied slots 0..U-1 (any order).  Each thread counts its grid-stride slots, the block scans the
// counts in LDS and reserves its range with ONE counter add (a single counter hit once per wave took 0.37 ms at
// 32k waves), then the threads walk the same slots again handing out base + prefix.
__global__ __launch_bounds__(256) void smooth_hash_number(SmoothHash h, long cap) {
    __shared__ int scan[256];
    __shared__ int base;
    const long stride = (long)gridDim.x * 256;
    const long p0 = (long)blockIdx.x * 256 + threadIdx.x;
    int cnt = 0;
    for (long p = p0; p < cap; p += stride) cnt += h.keys[p] != SM_EMPTY;
    scan[threadIdx.x] = cnt;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan
        const int v = threadIdx.x >= o ? scan[threadIdx.x - o] : 0;
        __syncthreads();
        scan[threadIdx.x] += v;
        __syncthreads();
    }
    if (threadIdx.x == 255) base = scan[255] ? atomicAdd(h.count, scan[255]) : 0;
    __syncthreads();
    int idx = base + scan[threadIdx.x] - cnt;
    for (long p = p0; p < cap; p += stride) {
        const unsigned long long k = h.keys[p];
        if (k == SM_EMPTY) continue;
        h.vals[p] = idx;
        h.u_tile[idx] = (int)(k >> 32);
        h.u_pal[idx] = (int)((k >> 2) & 0x3FFFFFFFu);
        h.u_flags[idx] = (uint8_t)(((k & 2) ? PSYV_HMIRROR : 0) | ((k & 1) ? PSYV_VMIRROR : 0));
        idx++;
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

// The chain with SM_G lanes per position (SM_PW positions per one-wave block).  The previous item's descriptor stays
// in registers across steps (it is always either the old previous or the old current one), so a step reads only the
// current item's row: each lane loads its 192 / SM_G dimensions, forms the squared differences (each term rounded
// as in the reference, fp contraction off) into LDS, and the group's first lane adds the 192 terms in index order --
// the reference's sequential fp64 sum, bit for bit.  Decisions are uniform per group; the first lane writes.
constexpr int SM_G = 8, SM_PW = 64 / SM_G, SM_D2 = 96 / SM_G;  // double2 per lane
__global__ __launch_bounds__(64) void smooth_chain_coop_kernel(SmoothArgs a) {
    __shared__ double2 terms[SM_PW][96];
    const double inv = 1.0 / (64.0 * 3.0);  // cSqrtFactor main.pas:4073
    const int lane = threadIdx.x, g = lane % SM_G, pw = lane / SM_G;
    const long s = (long)blockIdx.x * SM_PW + pw;
    const bool valid = s < a.Q;
    const long sq = valid ? s : 0;
    int pt = a.tile[sq], pp = a.pal[sq], ph = a.hm[sq], pv = a.vm[sq];
    int ptmp = a.tmpidx ? a.tmpidx[sq] : 0;
    double2 prev[SM_D2], cur[SM_D2], nxt[SM_D2];
    auto row = [&](int i) { return reinterpret_cast<const double2 *>(a.desc + (long)a.didx[(long)i * a.Q + sq] * 192) + g * SM_D2; };
    {
        const double2 *r = row(0);
#pragma unroll
        for (int j = 0; j < SM_D2; j++) prev[j] = r[j];
        if (a.F > 1) {
            const double2 *r1 = row(1);
#pragma unroll
            for (int j = 0; j < SM_D2; j++) nxt[j] = r1[j];
        }
    }
    for (int i = 1; i < a.F; i++) {  // uniform over the block: every group walks the same frames
        const long c = (long)i * a.Q + sq, p = (long)(i - 1) * a.Q + sq;
        const int ct = a.tile[c], cpl = a.pal[c], chm = a.hm[c], cvm = a.vm[c], csm = a.sm[c];
        const int ctmp = a.tmpidx ? a.tmpidx[c] : 0;
#pragma unroll
        for (int j = 0; j < SM_D2; j++) cur[j] = nxt[j];
        if (i + 1 < a.F) {  // the next frame's row does not depend on this step's decision: in flight across it
            const double2 *r = row(i + 1);
#pragma unroll
            for (int j = 0; j < SM_D2; j++) nxt[j] = r[j];
        }
#pragma unroll
        for (int j = 0; j < SM_D2; j++) {  // cur - prev, squared, every op rounded
            const double t0 = cur[j].x - prev[j].x, t1 = cur[j].y - prev[j].y;
            terms[pw][g * SM_D2 + j] = make_double2(t0 * t0, t1 * t1);
        }
        __syncthreads();
        double acc = 0.0;
        if (g == 0) {
#pragma unroll 8
            for (int k = 0; k < 96; k++) {
                const double2 v = terms[pw][k];
                acc += v.x;
                acc += v.y;
            }
        }
        __syncthreads();  // terms are rewritten next step
        acc = __shfl(acc, lane - g, 64);
        const double cmp = sqrt(acc * inv);
        const bool w = valid && g == 0;
        if (fabs(cmp) <= a.strength) {
            if (ct >= pt) {  // TMI^ := PrevTMI^ ; TMI^.Smoothed := True (prev item and descriptor unchanged)
                if (w) {
                    a.tile[c] = pt;
                    a.pal[c] = pp;
                    a.hm[c] = (uint8_t)ph;
                    a.vm[c] = (uint8_t)pv;
                    a.sm[c] = 1;
                    if (a.tmpidx) a.tmpidx[c] = ptmp;
                }
            } else {  // PrevTMI^ := TMI^ ; TMI^.Smoothed := True
                if (w) {
                    a.tile[p] = ct;
                    a.pal[p] = cpl;
                    a.hm[p] = (uint8_t)chm;
                    a.vm[p] = (uint8_t)cvm;
                    a.sm[p] = (uint8_t)csm;
                    if (a.tmpidx) a.tmpidx[p] = ctmp;
                    a.sm[c] = 1;
                }
                pt = ct, pp = cpl, ph = chm, pv = cvm, ptmp = ctmp;
#pragma unroll
                for (int j = 0; j < SM_D2; j++) prev[j] = cur[j];
            }
        } else {
            if (w) a.sm[c] = 0;
            pt = ct, pp = cpl, ph = chm, pv = cvm, ptmp = ctmp;
#pragma unroll
            for (int j = 0; j < SM_D2; j++) prev[j] = cur[j];
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
        {
            KTimer tk("smooth_hash", stream);
            hipLaunchKernelGGL(smooth_hash_insert, dim3(g), dim3(256), 0, stream, n, tile, pal, hm, vm, h);
            hipLaunchKernelGGL(smooth_hash_number, dim3((unsigned)std::min<long>(1024, (cap + 255) / 256)), dim3(256),
                               0, stream, h, cap);
            hipLaunchKernelGGL(smooth_hash_lookup, dim3(g), dim3(256), 0, stream, n, tile, pal, hm, vm, h);
        }
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
        pa.flags_per_mirrors_only = true;
        pa.flags = PSYV_FROM_PAL | PSYV_QWEIGHT;
        pa.gamma = -1;
        pa.out64 = desc;
        {
            KTimer tk("smooth_desc", stream);
            if (launch_psyv(pa, stream)) break;
        }
        SmoothArgs a{F, Q, tile, tmpidx, pal, hm, vm, sm, h.didx, desc, strength};
        // SM_G lanes per position, one wave per block
        KTimer tk("smooth_chain", stream);
        hipLaunchKernelGGL(smooth_chain_coop_kernel, dim3((unsigned)((Q + SM_PW - 1) / SM_PW)), dim3(64), 0, stream, a);
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

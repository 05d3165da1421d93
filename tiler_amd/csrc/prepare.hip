// prepare.hip -- PrepareFrameTiling (main.pas:3791-3967) for one keyframe on the device.
//
// The reference walks the keyframe's tilemap items on the host (UseOne per distinct (PalIdx, GlobalTileIndex),
// ProcThreadPool), searches each item's 64 palette indices k = 8 in FGlobalDS's kd-tree (main.pas:3830), marks
// used[pal', tile', attr] (3832-3852), emits the used cells' descriptors in DoPsyV order (3883-3919) and builds the
// keyframe's kd-tree (3961).  Here every step is a device pass over the keyframe at once, integer / byte work:
//   pf_bits_kernel        items -> a bitmap over the P*T (pal, tile) keys (atomic OR): distinct items, in key order
//   pf_bm_count/scan/place  bitmap compaction (block popcounts, one scan, ordered placement; no sort)
//   pf_qrows_kernel       the distinct items' query lines (palette indices as fp32)
//   nn_search_dev(k = 8)  the exact k = 8 search in ANN's tie order (nn_search.hip)
//   pf_mark_kernel        UseOne's walk of the 8 results (equal err after the first skipped) -> used bitmap
//                         [P][T][4], for the item's palette (Fast), the palettes near it (Medium), all (Slow)
//   pf_bm_* (cells)       used cells in (palette, tile, vmir, hmir) order = DoPsyV's emission order -> TRTo* maps
// then the candidate descriptors (psyv) and the keyframe's index (orbit grouping + ANN kd-tree).
#include <algorithm>

#include "prepare.hpp"
#include "psyv.hpp"

namespace tiler {

__global__ __launch_bounds__(256) void pf_bits_kernel(const int32_t *__restrict__ tile, const int32_t *__restrict__ pal,
                                                      long n, int T, int P, unsigned *bits) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const int t = tile[i], p = pal[i];
        if ((unsigned)t >= (unsigned)T || (unsigned)p >= (unsigned)P) continue;  // no item (-1) / out of range
        const long key = (long)p * T + t;
        atomicOr(bits + (key >> 5), 1u << (key & 31));
    }
}

// block = 256 words: its set-bit count
__global__ __launch_bounds__(256) void pf_bm_count_kernel(const unsigned *__restrict__ bits, long nwords, int *bcnt) {
    __shared__ int ws[4];
    const long w = (long)blockIdx.x * 256 + threadIdx.x;
    int c = w < nwords ? __popc(bits[w]) : 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// exclusive prefix of the block counts (one workgroup); total -> *total
__global__ __launch_bounds__(1024) void pf_scan_kernel(int *bcnt, int nb, int *total) {
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
        if (b < nb) bcnt[b] = carry + sc[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += sc[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// set bits of the bitmap in ascending order: key (= bit index) -> out[rank].  MODE 0: out_key[rank] = key.
// MODE 1 (the used cells p*T*4 + t*4 + a): the DoPsyV dataset maps + psyv mirror flags.
struct CellOut {
    int32_t *tile_of, *pal_of;
    uint8_t *attrs, *flags;
    const uint8_t *thm, *tvm;
    int T;
};
template <int MODE>
__global__ __launch_bounds__(256) void pf_bm_place_kernel(const unsigned *__restrict__ bits, long nwords,
                                                          const int *__restrict__ boff, int *out_key, CellOut co) {
    __shared__ int sc[256];
    const long w = (long)blockIdx.x * 256 + threadIdx.x;
    unsigned v = w < nwords ? bits[w] : 0u;
    const int c = __popc(v);
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int u = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
        __syncthreads();
        sc[threadIdx.x] += u;
        __syncthreads();
    }
    long r = (long)boff[blockIdx.x] + sc[threadIdx.x] - c;
    while (v) {
        const int b = __builtin_ctz(v);
        v &= v - 1;
        const long key = w * 32 + b;
        if (MODE == 0) {
            out_key[r] = (int)key;
        } else {
            const long cell = key >> 2;  // p * T + t
            const int a = (int)(key & 3);
            const int t = (int)(cell % co.T), p = (int)(cell / co.T);
            co.tile_of[r] = t;
            co.pal_of[r] = p;
            co.attrs[r] = (uint8_t)a;  // hm | vm << 1 (TRToAttrs, main.pas:3916)
            // the mirror DoPsyV applies: (hmir xor T.HMirror, vmir xor T.VMirror) (main.pas:3912)
            co.flags[r] = (uint8_t)((((a & 1) ^ co.thm[t]) ? PSYV_HMIRROR : 0) | ((((a >> 1) & 1) ^ co.tvm[t]) ? PSYV_VMIRROR : 0));
        }
        r++;
    }
}

__global__ __launch_bounds__(256) void pf_qrows_kernel(const int *__restrict__ keys, long nq, int T,
                                                       const uint8_t *__restrict__ palpix, float *qrows) {
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < nq * 64; e += (long)gridDim.x * 256) {
        const long i = e >> 6;
        const int t = keys[i] % T;
        qrows[e] = (float)palpix[(long)t * 64 + (e & 63)];
    }
}

// UseOne (main.pas:3830-3852): result j of item i is taken unless its err equals result j-1's (the reference keeps
// the last err it saw, starting from +inf) or it does not exist; the cell (tile', attr) of the global dataset row is
// marked for the palettes the quality selects.  Every write sets a bit to 1, so the races are benign.
__global__ __launch_bounds__(256) void pf_mark_kernel(const int *__restrict__ keys, long nq, int T, int P,
                                                      const int *__restrict__ idx, const float *__restrict__ err,
                                                      const int32_t *__restrict__ tr_tile,
                                                      const uint8_t *__restrict__ tr_attr, int quality,
                                                      const uint8_t *__restrict__ near, unsigned *used) {
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < nq * 8; e += (long)gridDim.x * 256) {
        const long i = e >> 3;
        const int j = (int)(e & 7);
        const float ej = err[e];
        if (j > 0 && ej == err[e - 1]) continue;  // (j = 0: the previous err is +inf, never equal)
        const int r = idx[e];
        if (r < 0) continue;
        const long cell = (long)tr_tile[r] * 4 + tr_attr[r];
        const int p = keys[i] / T;
        auto mark = [&](int pp) {
            const long bit = (long)pp * T * 4 + cell;
            atomicOr(used + (bit >> 5), 1u << (bit & 31));
        };
        if (quality == 0) {
            mark(p);
        } else {
            for (int pp = 0; pp < P; pp++)
                if (quality == 2 || near[(long)pp * P + p]) mark(pp);
        }
    }
}

template <typename T>
static int grow(T *&p, size_t &cap, size_t need) {
    if (need <= cap) return 0;
    hipFree(p);
    p = nullptr;
    cap = 0;
    TILER_HIP_CHECK(hipMalloc((void **)&p, std::max<size_t>(need, 1) * sizeof(T)));
    cap = need;
    return 0;
}

void prep_scratch_free(PrepScratch *s) {
    if (!s) return;
    hipFree(s->bits);
    hipFree(s->bcnt);
    hipFree(s->total);
    hipFree(s->keys);
    hipFree(s->qrows);
    hipFree(s->nn_idx);
    hipFree(s->nn_err);
    hipFree(s->near);
    hipFree(s->used);
    hipFree(s->tile_of);
    hipFree(s->pal_of);
    hipFree(s->attrs);
    hipFree(s->flags);
    hipHostFree(s->h_total);
    if (s->done) hipEventDestroy(s->done);
    *s = PrepScratch{};
}

// bitmap compaction: counts + scan (device total in *total), returns after the launches (no sync)
static int bm_scan(const unsigned *bits, long nwords, PrepScratch &s, int *total, hipStream_t stream) {
    const long nb = (nwords + 255) / 256;
    size_t cap = s.cap_blk;
    if (grow(s.bcnt, cap, (size_t)nb)) return -1;
    s.cap_blk = cap;
    hipLaunchKernelGGL(pf_bm_count_kernel, dim3((unsigned)nb), dim3(256), 0, stream, bits, nwords, s.bcnt);
    hipLaunchKernelGGL(pf_scan_kernel, dim3(1), dim3(1024), 0, stream, s.bcnt, (int)nb, total);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

NNIndex *prepare_frame_tiling_dev(NNIndex *global, PrepScratch &s, const int32_t *d_item_tile,
                                  const int32_t *d_item_pal, long n_items, const uint8_t *d_palpix,
                                  const uint8_t *d_thm, const uint8_t *d_tvm, int T, const int32_t *d_palettes, int P,
                                  int quality, const uint8_t *h_near, int use_wavelets, int gamma, hipStream_t stream,
                                  long *n_distinct, long *n_cand) {
    if (!global || global->d != 64 || !global->d_tr_tile || !global->d_tr_attr) {
        set_error("prepare_frame_tiling: the global dataset must be PrepareGlobalFT's 64-d rows with maps set");
        return nullptr;
    }
    if (T <= 0 || P <= 0 || n_items < 0 || (long)P * T * 4 >= (1L << 31) || quality < 0 || quality > 2 ||
        (quality == 1 && !h_near)) {
        set_error("prepare_frame_tiling: invalid arguments");
        return nullptr;
    }
    if (!s.h_total) TILER_HIP_CHECK_NULL(hipHostMalloc((void **)&s.h_total, 2 * sizeof(int), hipHostMallocPortable));
    if (!s.total) TILER_HIP_CHECK_NULL(hipMalloc((void **)&s.total, 2 * sizeof(int)));
    if (!s.done) TILER_HIP_CHECK_NULL(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    // the previous prepare's map copies (queued on its own stream) still read tile_of / pal_of / attrs
    TILER_HIP_CHECK_NULL(hipStreamWaitEvent(stream, s.done, 0));
    // 1. distinct (pal, tile) items in key order
    const long nkw = ((long)P * T + 31) / 32;
    const long nuw = ((long)P * T * 4 + 31) / 32;
    if (grow(s.bits, s.cap_bits, (size_t)nkw)) return nullptr;
    if (grow(s.used, s.cap_used, (size_t)nuw * 4)) return nullptr;  // bytes: the used-cell bitmap
    TILER_HIP_CHECK_NULL(hipMemsetAsync(s.bits, 0, (size_t)nkw * 4, stream));
    if (n_items > 0)
        hipLaunchKernelGGL(pf_bits_kernel, dim3((unsigned)std::min<long>(4096, (n_items + 255) / 256)), dim3(256), 0,
                           stream, d_item_tile, d_item_pal, n_items, T, P, s.bits);
    if (bm_scan(s.bits, nkw, s, s.total, stream)) return nullptr;
    TILER_HIP_CHECK_NULL(hipMemcpyAsync(s.h_total, s.total, sizeof(int), hipMemcpyDeviceToHost, stream));
    TILER_HIP_CHECK_NULL(hipStreamSynchronize(stream));
    const long nq = s.h_total[0];
    if ((size_t)nq > s.cap_items) {  // keys, query lines, k = 8 results: one capacity
        size_t c = 0;
        if (grow(s.keys, c, (size_t)nq)) return nullptr;
        c = 0;
        if (grow(s.qrows, c, (size_t)nq * 64)) return nullptr;
        c = 0;
        if (grow(s.nn_idx, c, (size_t)nq * 8)) return nullptr;
        c = 0;
        if (grow(s.nn_err, c, (size_t)nq * 8)) return nullptr;
        s.cap_items = nq;
    }
    hipLaunchKernelGGL((pf_bm_place_kernel<0>), dim3((unsigned)((nkw + 255) / 256)), dim3(256), 0, stream, s.bits,
                       nkw, s.bcnt, s.keys, CellOut{});
    TILER_HIP_CHECK_NULL(hipGetLastError());
    // 2. UseOne's k = 8 searches (exact, ANN's tie order) and the used bitmap
    if (quality == 1) {
        if (grow(s.near, s.cap_near, (size_t)P * P)) return nullptr;
        TILER_HIP_CHECK_NULL(hipMemcpyAsync(s.near, h_near, (size_t)P * P, hipMemcpyHostToDevice, stream));
    }
    unsigned *used = reinterpret_cast<unsigned *>(s.used);
    TILER_HIP_CHECK_NULL(hipMemsetAsync(used, 0, (size_t)nuw * 4, stream));
    if (nq > 0) {
        hipLaunchKernelGGL(pf_qrows_kernel, dim3((unsigned)std::min<long>(8192, (nq * 64 + 255) / 256)), dim3(256), 0,
                           stream, s.keys, nq, T, d_palpix, s.qrows);
        if (global->n > 0) {
            if (nn_search_dev(global, s.qrows, (int)nq, 8, s.nn_idx, s.nn_err, nullptr, stream)) return nullptr;
            hipLaunchKernelGGL(pf_mark_kernel, dim3((unsigned)std::min<long>(8192, (nq * 8 + 255) / 256)), dim3(256), 0,
                               stream, s.keys, nq, T, P, s.nn_idx, s.nn_err, global->d_tr_tile, global->d_tr_attr,
                               quality, s.near, used);
        }
    }
    // 3. the used cells in DoPsyV's emission order
    if (bm_scan(used, nuw, s, s.total + 1, stream)) return nullptr;
    TILER_HIP_CHECK_NULL(hipMemcpyAsync(s.h_total + 1, s.total + 1, sizeof(int), hipMemcpyDeviceToHost, stream));
    TILER_HIP_CHECK_NULL(hipStreamSynchronize(stream));
    const long M = s.h_total[1];
    if ((size_t)M > s.cap_cand) {
        size_t c = 0;
        if (grow(s.tile_of, c, (size_t)M)) return nullptr;
        c = 0;
        if (grow(s.pal_of, c, (size_t)M)) return nullptr;
        c = 0;
        if (grow(s.attrs, c, (size_t)M)) return nullptr;
        c = 0;
        if (grow(s.flags, c, (size_t)M)) return nullptr;
        s.cap_cand = M;
    }
    CellOut co{s.tile_of, s.pal_of, s.attrs, s.flags, d_thm, d_tvm, T};
    hipLaunchKernelGGL((pf_bm_place_kernel<1>), dim3((unsigned)((nuw + 255) / 256)), dim3(256), 0, stream, used, nuw,
                       s.bcnt, nullptr, co);
    TILER_HIP_CHECK_NULL(hipGetLastError());
    // 4. DoPsyV: the candidates' descriptors (fp64 -> fp32 rows), then the keyframe's index
    float *rows = nullptr;
    TILER_HIP_CHECK_NULL(dmalloc((void **)&rows, (size_t)std::max<long>(M, 1) * 192 * sizeof(float)));  // the index owns it
    PsyvArgs pa;
    pa.n = M;
    pa.palpix = d_palpix;
    pa.tile_of = s.tile_of;
    pa.palettes = d_palettes;
    pa.pal_of = s.pal_of;
    pa.flags_per = s.flags;
    pa.flags_per_mirrors_only = true;
    pa.flags = PSYV_FROM_PAL | (use_wavelets ? PSYV_WAVELETS : 0);
    pa.gamma = gamma;
    pa.out32 = rows;
    if (M > 0 && launch_psyv(pa, stream)) {
        hipFree(rows);
        return nullptr;
    }
    NNIndex *ix = nn_index_create_dev(rows, (int)M, 192, 1, KD_SPLIT_STD, stream);  // owns rows
    if (!ix) return nullptr;
    const size_t n1 = std::max<long>(M, 1);
    if (dmalloc((void **)&ix->d_tr_tile, n1 * 4) != hipSuccess || dmalloc((void **)&ix->d_tr_pal, n1 * 4) != hipSuccess ||
        dmalloc((void **)&ix->d_tr_attr, n1) != hipSuccess ||
        hipMemcpyAsync(ix->d_tr_tile, s.tile_of, (size_t)M * 4, hipMemcpyDeviceToDevice, stream) != hipSuccess ||
        hipMemcpyAsync(ix->d_tr_pal, s.pal_of, (size_t)M * 4, hipMemcpyDeviceToDevice, stream) != hipSuccess ||
        hipMemcpyAsync(ix->d_tr_attr, s.attrs, (size_t)M, hipMemcpyDeviceToDevice, stream) != hipSuccess) {
        set_error("prepare_frame_tiling: map allocation failed");
        nn_index_destroy(ix);
        return nullptr;
    }
    TILER_HIP_CHECK_NULL(hipEventRecord(s.done, stream));
    if (n_distinct) *n_distinct = nq;
    if (n_cand) *n_cand = M;
    return ix;
}

}  // namespace tiler

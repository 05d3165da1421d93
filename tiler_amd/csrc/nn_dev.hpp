// nn_dev.hpp -- device helpers shared by the NN-search kernels (nn_search.hip, orbit.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

// the reference distance is a sequential fp32 sum with every op rounded: no FMA contraction anywhere
#pragma clang fp contract(off)

namespace tiler {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// one 16-byte LDS-DMA piece per lane: LDS destination = wave-uniform base + lane * 16
__device__ __forceinline__ void glds16(const uint4 *gsrc, char *lds_wave_base) {
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    __builtin_amdgcn_global_load_lds((gvoid *)(gsrc), (lvoid *)(lds_wave_base), 16, 0, 0);
}

// The same DMA as inline asm, invisible to hipcc's waitcnt pass: the compiler counts a pending
// global_load_lds as an LGKM event of another kind, which makes every later LDS-read wait an
// lgkmcnt(0) (no read can stay in flight behind an MFMA).  Users drain it themselves: dma_drain()
// before the barrier that publishes the stage.
__device__ __forceinline__ void glds16_asm(const uint4 *gsrc, char *lds_wave_base) {
    const unsigned lds = __builtin_amdgcn_readfirstlane(
        (unsigned)(size_t)(__attribute__((address_space(3))) char *)lds_wave_base);
    asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(gsrc), "{m0}"(lds) : "memory");
}
__device__ __forceinline__ void dma_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double wave_max_d(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

template <int L>
__device__ __forceinline__ void list_insert(float (&k)[L], int (&id)[L], float x, int ix) {
#pragma unroll
    for (int i = L - 1; i > 0; --i) {
        const bool gp = k[i - 1] > x, gc = k[i] > x;
        const float nk = gp ? k[i - 1] : (gc ? x : k[i]);
        const int ni = gp ? id[i - 1] : (gc ? ix : id[i]);
        k[i] = nk;
        id[i] = ni;
    }
    if (k[0] > x) {
        k[0] = x;
        id[0] = ix;
    }
}

// D = 192 (the FrameTiling descriptor): fully unrolled so every load is issued up front and only the
// reference's dependent add chain remains (the runtime-d loop below waits on a load per 4 terms)
__device__ __forceinline__ float exact_dist192(const float *__restrict__ q, const float *__restrict__ c) {
    const float4 *q4 = reinterpret_cast<const float4 *>(q), *c4 = reinterpret_cast<const float4 *>(c);
    float dist = 0.0f;
#pragma unroll
    for (int h = 0; h < 4; h++) {  // 4 chunks of 12 float4 each: loads of a chunk issued together
        float4 qa[12], ca[12];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            qa[i] = q4[h * 12 + i];
            ca[i] = c4[h * 12 + i];
        }
#pragma unroll
        for (int i = 0; i < 12; i++) {
            float t;
            t = qa[i].x - ca[i].x; dist = dist + t * t;
            t = qa[i].y - ca[i].y; dist = dist + t * t;
            t = qa[i].z - ca[i].z; dist = dist + t * t;
            t = qa[i].w - ca[i].w; dist = dist + t * t;
        }
    }
    return dist;
}

__device__ __forceinline__ float exact_dist(const float *__restrict__ q, const float *__restrict__ c, int d) {
    if (d == 192) return exact_dist192(q, c);
    float dist = 0.0f;
    int i = 0;
    if ((d & 3) == 0) {
        const float4 *q4 = reinterpret_cast<const float4 *>(q), *c4 = reinterpret_cast<const float4 *>(c);
        for (; i < d / 4; i++) {
            const float4 a = q4[i], b = c4[i];
            float t;
            t = a.x - b.x; dist = dist + t * t;
            t = a.y - b.y; dist = dist + t * t;
            t = a.z - b.z; dist = dist + t * t;
            t = a.w - b.w; dist = dist + t * t;
        }
        return dist;
    }
    for (; i < d; i++) {
        const float t = q[i] - c[i];
        dist = dist + t * t;
    }
    return dist;
}

// lexicographic (v, i) wave minimum
__device__ __forceinline__ void wave_argmin(float &v, int &i) {
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        const bool take = (ov < v) || (ov == v && (unsigned)oi < (unsigned)i);
        v = take ? ov : v;
        i = take ? oi : i;
    }
}

__device__ __forceinline__ bool lex_less(float a, int ia, float b, int ib) {
    return a < b || (a == b && (unsigned)ia < (unsigned)ib);
}

}  // namespace tiler

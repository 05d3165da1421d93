// psyv.hip -- PsyV tile descriptor on gfx950 (ComputeTilePsyVisFeatures, main.pas:2997-3177).
//
// One wave64 per 8x8 tile, lane = pixel (y*8+x) for the colour conversion and = output coefficient
// for the transform.  All arithmetic is fp64 in the reference's source order with no contraction,
// so results are bit-identical to the CPU restatement (oracle/tiler_oracle.c):
//   - RGBToYUV (main.pas:2656-2679) with r/255 and gGammaCorLut taken from a host-built LUT;
//   - WaveletGS (main.pas:2805-2840): 3 Haar levels, rows then columns, neighbours via ds_bpermute;
//   - DCT branch (main.pas:3075-3175): sequential 64-term sums against the host-built gDCTLut.
// HBM traffic per tile: 256 B in (RGB) or 64 B + 64 B palette, 768 B (fp32) / 1536 B (fp64) out.
#include "psyv.hpp"
#include "psyv_dev.hpp"

#pragma clang fp contract(off)

namespace tiler {

__global__ __launch_bounds__(256) void psyv_kernel(PsyvArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int y = lane >> 3, x = lane & 7;
    const double *__restrict__ glut = a.gamma_lut + 256 * (a.gamma + 1);
    for (long i = (long)blockIdx.x * 4 + wave; i < a.n; i += (long)gridDim.x * 4) {
        int f = a.flags | (a.flags_per ? a.flags_per[i] : 0);
        const int xx = (f & PSYV_HMIRROR) ? 7 - x : x;
        const int yy = (f & PSYV_VMIRROR) ? 7 - y : y;
        const int src = yy * 8 + xx;
        int32_t col;
        if (f & PSYV_FROM_PAL) {
            const long t = a.tile_of ? a.tile_of[i] : i;
            const long p = a.pal_of ? a.pal_of[i] : 0;
            col = a.palettes[p * 16 + a.palpix[t * 64 + src]];
        } else {
            col = a.rgb[i * 64 + src];
        }
        double cp[3];
        if (f & PSYV_LAB)
            lab_of(col, a.lab_lin + 256 * (a.gamma + 1), cp[0], cp[1], cp[2]);
        else
            yuv_of(col, glut, a.u_mul, a.v_mul, cp[0], cp[1], cp[2]);
        double out[3];
        if (f & PSYV_WAVELETS) {
#pragma unroll
            for (int c = 0; c < 3; c++) out[c] = haar3(cp[c], y, x, a.haar_f);
        } else {
            const PsyvConst k{a.gamma_lut, a.dct_lut, a.qmul, a.ratio, a.haar_f, a.u_mul, a.v_mul};
#pragma unroll
            for (int c = 0; c < 3; c++) out[c] = dct_lane(cp[c], lane, c, (f & PSYV_QWEIGHT) != 0, k);
        }
#pragma unroll
        for (int c = 0; c < 3; c++) {
            if (a.out64) a.out64[i * 192 + c * 64 + lane] = out[c];
            if (a.out32) a.out32[i * 192 + c * 64 + lane] = (float)out[c];
        }
    }
}

// FrameTiling query descriptors (RGB, no mirror, Haar: DoFrameTiling main.pas:4023): one LANE per tile, the
// whole 3-level WaveletGS of each component in registers (haar_regs, psyv_dev.hpp), gamma LUT in LDS.
template <bool FASTDIV>
__global__ __launch_bounds__(64) void psyv_rgb_haar_kernel(PsyvArgs a) {
    __shared__ double lut[256];
    __shared__ float st[64 * 65];  // one component of the 64 tiles, transposed for coalesced row stores
    __shared__ float sbox[2 * 192];
    const int lane = threadIdx.x;
    const double *__restrict__ glut = a.gamma_lut + 256 * (a.gamma + 1);
    for (int i = lane; i < 256; i += 64) lut[i] = glut[i];
    if (a.rootbox)
        for (int i = lane; i < 2 * 192; i += 64) sbox[i] = a.box[i];
    __syncthreads();
    float rb = 0.0f;  // annBoxDistance, accumulated in dimension order (c, k)
    const long t0 = (long)blockIdx.x * 64;
    const long i = t0 + lane;
    const bool valid = i < a.n;
    const long ti = valid ? i : t0;
    const int4 *src = reinterpret_cast<const int4 *>(a.rgb + (a.perm ? (long)a.perm[ti] : ti) * 64);
#pragma unroll 1
    for (int c = 0; c < 3; c++) {
        double p[64];
#pragma unroll
        for (int k4 = 0; k4 < 16; k4++) {
            const int4 v = src[k4];  // re-read per component (L1): keeps 64 colours out of the registers
            const int cc[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int r = cc[e] & 0xff, g = (cc[e] >> 8) & 0xff, b = (cc[e] >> 16) & 0xff;
                const double fr = lut[r], fg = lut[g], fb = lut[b];
                const double cy = div10000<FASTDIV>(2126.0 * fr + 7152.0 * fg + 722.0 * fb);
                p[4 * k4 + e] = c == 0 ? cy : c == 1 ? (fb - cy) * a.u_mul : (fr - cy) * a.v_mul;
            }
        }
        haar_regs(p, a.haar_f);
        if (a.rootbox) {
#pragma unroll
            for (int k = 0; k < 64; k++) {
                const float v = (float)p[k], lo = sbox[c * 64 + k], hi = sbox[192 + c * 64 + k];
                if (v < lo) {
                    const float t = lo - v;
                    rb = rb + t * t;
                } else if (v > hi) {
                    const float t = v - hi;
                    rb = rb + t * t;
                }
            }
        }
        if (a.out32) {
            // lane = tile: its 64 values into LDS (stride 65: conflict-free), then 16 lanes per tile store
            // the tile's 256-byte component segment (64-byte lines written whole, not a line per lane)
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 64; k++) st[lane * 65 + k] = (float)p[k];
            __syncthreads();
#pragma unroll
            for (int t = 0; t < 16; t++) {
                const int pc = lane + 64 * t, tt = pc >> 4, c4 = pc & 15;
                if (t0 + tt < a.n) {
                    const float *q = st + tt * 65 + c4 * 4;
                    reinterpret_cast<float4 *>(a.out32 + (t0 + tt) * 192 + c * 64)[c4] = make_float4(q[0], q[1], q[2], q[3]);
                }
            }
        }
        if (a.out64 && valid) {
            double2 *o = reinterpret_cast<double2 *>(a.out64 + i * 192 + c * 64);
#pragma unroll
            for (int k = 0; k < 32; k++) o[k] = make_double2(p[2 * k], p[2 * k + 1]);
        }
    }
    if (a.rootbox && valid) a.rootbox[i] = rb;
}

// DCT descriptors of palette tiles (the Smooth step's distinct items, main.pas:3075-3175 via 4097-4098) with ONE
// LANE per item: the lane's 64 colours (own palette, own mirrors) staged in LDS, one component's 64 fp64 values in
// registers, and each output o = sum_i cp_i * gDCTLut[o][i] summed in i order exactly as dct_lane does -- the LUT
// row is the same for every lane, so its operand comes through the scalar cache instead of 64 cross-lane
// shuffles per output.  Then the Q-weighting and the ratio, as dct_lane.
__global__ __launch_bounds__(64) void psyv_dct_items_kernel(PsyvArgs a) {
    __shared__ int32_t cols[64][65];
    const int lane = threadIdx.x;
    const long i = (long)blockIdx.x * 64 + lane;
    const bool valid = i < a.n;
    const long ii = valid ? i : 0;
    const int f = a.flags | (a.flags_per ? a.flags_per[ii] : 0);
    const int m = ((f & PSYV_HMIRROR) ? 7 : 0) ^ ((f & PSYV_VMIRROR) ? 56 : 0);  // source pixel = k ^ m
    const long t = a.tile_of ? a.tile_of[ii] : ii;
    const long p = a.pal_of ? a.pal_of[ii] : 0;
    const uint8_t *px = a.palpix + t * 64;
    const int32_t *pal = a.palettes + p * 16;
#pragma unroll 8
    for (int k = 0; k < 64; k++) cols[lane][k] = pal[px[k ^ m]];
    const double *__restrict__ glut = a.gamma_lut + 256 * (a.gamma + 1);
    const bool qw = (f & PSYV_QWEIGHT) != 0;
#pragma unroll 1
    for (int c = 0; c < 3; c++) {
        double cp[64];
#pragma unroll
        for (int k = 0; k < 64; k++) {
            double cy, cu, cv;
            yuv_of(cols[lane][k], glut, a.u_mul, a.v_mul, cy, cu, cv);
            cp[k] = c == 0 ? cy : c == 1 ? cu : cv;
        }
#pragma unroll 1
        for (int o = 0; o < 64; o++) {
            const double *__restrict__ L = a.dct_lut + o * 64;  // uniform: scalar loads
            double z = 0.0;
#pragma unroll
            for (int k = 0; k < 64; k++) z += cp[k] * L[k];
            if (qw) z *= a.qmul[c * 64 + o];
            z = z * a.ratio[o];
            if (valid) {
                if (a.out64) a.out64[i * 192 + c * 64 + o] = z;
                if (a.out32) a.out32[i * 192 + c * 64 + o] = (float)z;
            }
        }
    }
}

static constexpr long PSYV_LANE_ITEMS_MIN = 32768;  // C3 bench keyframe (~20k items): 0.04 ms wave-per-item vs 0.31

int launch_psyv(PsyvArgs args, hipStream_t stream) {
    if (args.n <= 0) return 0;
    const Luts &L = luts();
    args.gamma_lut = L.d_gamma;
    args.dct_lut = L.d_dct;
    args.qmul = L.d_qmul;
    args.ratio = L.d_ratio;
    args.lab_lin = L.d_lab_lin;
    args.haar_f = L.haar_f;
    args.u_mul = L.u_mul;
    args.v_mul = L.v_mul;
    if (args.gamma < -1 || args.gamma > 1) {
        set_error("psyv: gamma must be -1, 0 or 1");
        return -1;
    }
    KTimer tm("psyv", stream);
    if (args.rootbox && !(args.rgb && !args.flags_per && args.flags == PSYV_WAVELETS)) {
        set_error("psyv: the fused root-box output exists on the RGB Haar query path only");
        return -1;
    }
    if (args.perm && !(args.rgb && !args.flags_per && (args.flags & ~PSYV_QWEIGHT) == PSYV_WAVELETS)) {
        set_error("psyv: a query permutation exists on the RGB Haar query path only");
        return -1;
    }
    if (args.rgb && !args.flags_per && (args.flags & ~PSYV_QWEIGHT) == PSYV_WAVELETS) {
        const dim3 grid((unsigned)((args.n + 63) / 64));
        if (args.gamma == -1)
            hipLaunchKernelGGL(psyv_rgb_haar_kernel<true>, grid, dim3(64), 0, stream, args);
        else
            hipLaunchKernelGGL(psyv_rgb_haar_kernel<false>, grid, dim3(64), 0, stream, args);
    } else if ((args.flags & PSYV_FROM_PAL) && !(args.flags & (PSYV_WAVELETS | PSYV_LAB)) && !args.rgb &&
               (!args.flags_per || args.flags_per_mirrors_only) && args.n >= PSYV_LANE_ITEMS_MIN) {
        // many items: one lane each (a wave per item below this count: each lane's 12k-add chain would run alone)
        hipLaunchKernelGGL(psyv_dct_items_kernel, dim3((unsigned)((args.n + 63) / 64)), dim3(64), 0, stream, args);
    } else {
        long blocks = (args.n + 3) / 4;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(psyv_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, args);
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tiler

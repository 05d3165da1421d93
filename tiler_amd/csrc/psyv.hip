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

#pragma clang fp contract(off)

namespace tiler {

__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src, 64); }

// one Haar level on the dx x dx top-left block (WaveletGS body, main.pas:2818-2836)
__device__ __forceinline__ double haar_level(double d, int y, int x, int dx, double f) {
    const int half = dx >> 1;
    // rows: tempX[y][x] = (D[y][2x'] +/- D[y][2x'+1]) * f, x' = x mod half
    const int xs = x & (half - 1);
    double a = shfl_d(d, y * 8 + 2 * xs);
    double b = shfl_d(d, y * 8 + 2 * xs + 1);
    double tx = (x < half) ? (a + b) * f : (a - b) * f;
    // columns: tempY[y][x] = (tempX[2y'][x] +/- tempX[2y'+1][x]) * f, y' = y mod half
    const int ys = y & (half - 1);
    double c = shfl_d(tx, (2 * ys) * 8 + x);
    double e = shfl_d(tx, (2 * ys + 1) * 8 + x);
    double ty = (y < half) ? (c + e) * f : (c - e) * f;
    return (x < dx && y < dx) ? ty : d;
}

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
        const int r = col & 0xff, g = (col >> 8) & 0xff, b = (col >> 16) & 0xff;
        // RGBToYUV main.pas:2661-2676 (row 0 of the LUT is i/255.0 exactly as the host computes it)
        const double fr = glut[r], fg = glut[g], fb = glut[b];
        double cy = (2126.0 * fr + 7152.0 * fg + 722.0 * fb) / 10000.0;
        double cu = (fb - cy) * a.u_mul;
        double cv = (fr - cy) * a.v_mul;
        double cp[3] = {cy, cu, cv};
        double out[3];
        if (f & PSYV_WAVELETS) {
#pragma unroll
            for (int c = 0; c < 3; c++) {
                double d = cp[c];
                d = haar_level(d, y, x, 8, a.haar_f);
                d = haar_level(d, y, x, 4, a.haar_f);
                d = haar_level(d, y, x, 2, a.haar_f);
                out[c] = d;
            }
        } else {
            // lane = (v, u); z = sum_k cpn[k] * gDCTLut[(v*8+u)*64 + k], sequential (main.pas:3092-3167)
            const double *__restrict__ lut = a.dct_lut + lane * 64;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                double z = 0.0;
                for (int k = 0; k < 64; k++) z += shfl_d(cp[c], k) * lut[k];
                if (f & PSYV_QWEIGHT) z *= a.qmul[c * 64 + lane];
                out[c] = z * a.ratio[lane];
            }
        }
#pragma unroll
        for (int c = 0; c < 3; c++) {
            if (a.out64) a.out64[i * 192 + c * 64 + lane] = out[c];
            if (a.out32) a.out32[i * 192 + c * 64 + lane] = (float)out[c];
        }
    }
}

int launch_psyv(PsyvArgs args, hipStream_t stream) {
    if (args.n <= 0) return 0;
    const Luts &L = luts();
    args.gamma_lut = L.d_gamma;
    args.dct_lut = L.d_dct;
    args.qmul = L.d_qmul;
    args.ratio = L.d_ratio;
    args.haar_f = L.haar_f;
    args.u_mul = L.u_mul;
    args.v_mul = L.v_mul;
    if (args.gamma < -1 || args.gamma > 1) {
        set_error("psyv: gamma must be -1, 0 or 1");
        return -1;
    }
    long blocks = (args.n + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    KTimer tm("psyv", stream);
    hipLaunchKernelGGL(psyv_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, args);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tiler

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

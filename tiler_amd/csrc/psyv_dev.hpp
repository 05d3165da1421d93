// psyv_dev.hpp -- wave64 device helpers for the PsyV descriptor (shared by psyv.hip and smooth.hip).
// Lane = pixel (y*8+x) for the colour conversion, = output coefficient for the transform.
// fp64 throughout in the reference's source order; the including file sets fp contract(off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "detmath.hpp"

namespace tiler {

struct PsyvConst {
    const double *gamma_lut;  // [3][256]
    const double *dct_lut;    // [4096]
    const double *qmul;       // [192]
    const double *ratio;      // [64]
    double haar_f, u_mul, v_mul;
};

__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src, 64); }

// RGBToYUV main.pas:2656-2679; glut = gGammaCorLut row (row 0 = i/255.0 exactly as the host computes it)
__device__ __forceinline__ void yuv_of(int32_t col, const double *__restrict__ glut, double u_mul, double v_mul,
                                       double &cy, double &cu, double &cv) {
    const int r = col & 0xff, g = (col >> 8) & 0xff, b = (col >> 16) & 0xff;
    const double fr = glut[r], fg = glut[g], fb = glut[b];
    cy = (2126.0 * fr + 7152.0 * fg + 722.0 * fb) / 10000.0;
    cu = (fb - cy) * u_mul;
    cv = (fr - cy) * v_mul;
}

// RGBToLAB main.pas:2711-2747 (UseLAB: the Dither step's descriptors); lin = the gamma row of the host-built
// linearised-channel LUT (main.pas:2715-2721), the cube roots are FPC power = exp(ln(t) / 3) (detmath.hpp)
__device__ __forceinline__ void lab_of(int32_t col, const double *__restrict__ lin, double &ol, double &oa,
                                       double &ob) {
    const double r = lin[col & 0xff], g = lin[(col >> 8) & 0xff], b = lin[(col >> 16) & 0xff];
    double x = (r * 0.49000 + g * 0.31000 + b * 0.20000) / 0.17697;
    double y = (r * 0.17697 + g * 0.81240 + b * 0.01063) / 0.17697;
    double z = (r * 0.00000 + g * 0.01000 + b * 0.99000) / 0.17697;
    x /= 96.6797 / 100;  // illuminant D50
    y /= 100.000 / 100;
    z /= 82.5188 / 100;
    x = x > 0.008856 ? fpc_power_frac(x, 1.0 / 3.0) : (7.787 * x) + 16.0 / 116.0;
    y = y > 0.008856 ? fpc_power_frac(y, 1.0 / 3.0) : (7.787 * y) + 16.0 / 116.0;
    z = z > 0.008856 ? fpc_power_frac(z, 1.0 / 3.0) : (7.787 * z) + 16.0 / 116.0;
    ol = (116 * y) - 16;
    oa = 500 * (x - y);
    ob = 200 * (y - z);
}

// one WaveletGS level on the dx x dx top-left block (main.pas:2818-2836)
__device__ __forceinline__ double haar_level(double d, int y, int x, int dx, double f) {
    const int half = dx >> 1;
    const int xs = x & (half - 1);
    const double a = shfl_d(d, y * 8 + 2 * xs);
    const double b = shfl_d(d, y * 8 + 2 * xs + 1);
    const double tx = (x < half) ? (a + b) * f : (a - b) * f;
    const int ys = y & (half - 1);
    const double c = shfl_d(tx, (2 * ys) * 8 + x);
    const double e = shfl_d(tx, (2 * ys + 1) * 8 + x);
    const double ty = (y < half) ? (c + e) * f : (c - e) * f;
    return (x < dx && y < dx) ? ty : d;
}

__device__ __forceinline__ double haar3(double d, int y, int x, double f) {
    d = haar_level(d, y, x, 8, f);
    d = haar_level(d, y, x, 4, f);
    return haar_level(d, y, x, 2, f);
}

// DCT branch main.pas:3075-3175 for output (v,u) = lane of component c: sequential 64-term sum
__device__ __forceinline__ double dct_lane(double cp, int lane, int c, bool qweight, const PsyvConst &k) {
    const double *__restrict__ lut = k.dct_lut + lane * 64;
    double z = 0.0;
    for (int i = 0; i < 64; i++) z += shfl_d(cp, i) * lut[i];
    if (qweight) z *= k.qmul[c * 64 + lane];
    return z * k.ratio[lane];
}

// The 3-level WaveletGS of one 8x8 component held by ONE lane (compile-time indices, no cross-lane traffic):
// the same fp64 operations in the same order as haar3 / the CPU restatement.
__device__ __forceinline__ void haar_regs(double (&p)[64], double f) {
#pragma unroll
    for (int dx = 8; dx >= 2; dx >>= 1) {
        const int h = dx >> 1;
#pragma unroll
        for (int y = 0; y < dx; y++) {  // rows: L at x, H at x + dx/2
            double t[8];
#pragma unroll
            for (int x = 0; x < h; x++) {
                const double a = p[y * 8 + 2 * x], b = p[y * 8 + 2 * x + 1];
                t[x] = (a + b) * f;
                t[x + h] = (a - b) * f;
            }
#pragma unroll
            for (int x = 0; x < dx; x++) p[y * 8 + x] = t[x];
        }
#pragma unroll
        for (int x = 0; x < dx; x++) {  // columns
            double t[8];
#pragma unroll
            for (int y = 0; y < h; y++) {
                const double a = p[(2 * y) * 8 + x], b = p[(2 * y + 1) * 8 + x];
                t[y] = (a + b) * f;
                t[y + h] = (a - b) * f;
            }
#pragma unroll
            for (int y = 0; y < dx; y++) p[y * 8 + x] = t[y];
        }
    }
}

// x / 10000.0 for the gamma = -1 colour sums (fr = r / 255.0): q0 = x * RN(1e-4) plus one fma residual
// correction.  Bit-identical to the IEEE division over every (r, g, b) of the domain (all 2^24 sums checked
// by oracle/check_fastdiv.c, tests/test_oracle_kats.py); other gamma LUTs keep the true division.
// r / 255.0 for a byte r (the gamma = -1 row of gGammaCorLut, main.pas:606) without a LUT read: q0 = r * RN(1/255)
// plus one fma residual correction, bit-identical to the IEEE division for all 256 bytes
// (tests/test_oracle_kats.py::test_div255_identity).  Lets the FrameTiling query kernel skip its LDS gathers.
__device__ __forceinline__ double div255(int r) {
    const double x = (double)r, inv = 1.0 / 255.0;
    const double q0 = x * inv;
    return __builtin_fma(__builtin_fma(-q0, 255.0, x), inv, q0);
}

template <bool FASTDIV>
__device__ __forceinline__ double div10000(double x) {
    if constexpr (FASTDIV) {
        const double inv = 1.0 / 10000.0;
        const double q0 = x * inv;
        return __builtin_fma(__builtin_fma(-q0, 10000.0, x), inv, q0);
    } else {
        return x / 10000.0;
    }
}


}  // namespace tiler

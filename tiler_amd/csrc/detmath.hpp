// detmath.hpp -- deterministic exp / ln for host and device: the same IEEE double operations in the same order on
// both, so a value computed on the GPU equals the one the host (and the CPU restatement) computes.
//
// Used where the reference calls FPC's Math.power with a non-integer exponent, which FPC evaluates as
// exp(exponent * ln(base)): the LAB conversion of the Dither step's descriptors (RGBToLAB main.pas:2711-2747, via
// ComputeTilePsyVisFeatures(UseLAB) from PrepareDitherTiles main.pas:2120).  exp and ln follow the published
// fdlibm algorithms (e_exp.c: reduction by ln2 halves + degree-5 Remez polynomial; e_log.c: reduction to
// [sqrt(2)/2, sqrt(2)] + s = f / (2 + f) series); FPC's own RTL implementation is not part of the reference, so
// agreement with the reference binary is unpinned.  Compile with contraction off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tiler {

__host__ __device__ inline uint32_t dm_hi(double x) { return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
__host__ __device__ inline uint32_t dm_lo(double x) { return (uint32_t)__builtin_bit_cast(uint64_t, x); }
__host__ __device__ inline double dm_with_hi(double x, uint32_t hi) {
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | dm_lo(x));
}

// ln(x) (fdlibm e_log.c)
__host__ __device__ inline double det_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double two54 = 1.80143985094819840000e+16;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    int32_t hx = (int32_t)dm_hi(x);
    const uint32_t lx = dm_lo(x);
    int k = 0;
    if (hx < 0x00100000) {  // x < 2^-1022
        if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf();
        if (hx < 0) return __builtin_nan("");
        k -= 54;
        x *= two54;
        hx = (int32_t)dm_hi(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;
    x = dm_with_hi(x, (uint32_t)(hx | (i0 ^ 0x3ff00000)));  // normalise x or x / 2
    k += (i0 >> 20);
    const double f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            const double dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        const double dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    int32_t i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// e^x (fdlibm e_exp.c)
__host__ __device__ inline double det_exp(double x) {
    const double o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02;
    const double ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01};
    const double ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10};
    const double invln2 = 1.44269504088896338700e+00, halF[2] = {0.5, -0.5};
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
                 P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
    const double twom1000 = 9.33263618503218878990e-302;
    uint32_t hx = dm_hi(x);
    const int xsb = (int)((hx >> 31) & 1);
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {  // |x| >= 709.78...
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | dm_lo(x)) != 0) return x + x;  // NaN
            return xsb == 0 ? x : 0.0;                           // exp(+-inf)
        }
        if (x > o_threshold) return __builtin_inf();
        if (x < u_threshold) return 0.0;
    }
    double hi = 0.0, lo = 0.0;
    int k = 0;
    if (hx > 0x3fd62e42) {    // |x| > 0.5 ln2
        if (hx < 0x3FF0A2B2) {  // and |x| < 1.5 ln2
            hi = x - ln2HI[xsb];
            lo = ln2LO[xsb];
            k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + halF[xsb]);
            const double t = (double)k;
            hi = x - t * ln2HI[0];  // t * ln2HI is exact here
            lo = t * ln2LO[0];
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {  // |x| < 2^-28
        return 1.0 + x;
    } else {
        k = 0;
    }
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) return dm_with_hi(y, dm_hi(y) + ((uint32_t)k << 20));
    return dm_with_hi(y, dm_hi(y) + ((uint32_t)(k + 1000) << 20)) * twom1000;
}

// FPC Math.power(base, exponent) for the non-integer exponents the LAB conversion uses (2.4, 1/3):
// exp(exponent * ln(base)).  (Integer exponents go through FPC's intpower; no caller here needs them.)
__host__ __device__ inline double fpc_power_frac(double base, double exponent) {
    if (exponent == 0.0) return 1.0;
    if (base == 0.0 && exponent > 0.0) return 0.0;
    return det_exp(exponent * det_log(base));
}

}  // namespace tiler

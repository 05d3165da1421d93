/*
 * detmath.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * exp / ln as the published fdlibm algorithms (e_exp.c, e_log.c) in plain IEEE double arithmetic, and FPC
 * Math.power for non-integer exponents (exp(exponent * ln(base))), for the LAB conversion of the Dither step's
 * descriptors (RGBToLAB main.pas:2711-2747).  FPC's RTL implementation of exp / ln is not in the reference:
 * agreement with the reference binary is unpinned; the GPU product (tiler_amd/csrc/detmath.hpp) must equal this.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "tiler_oracle.h"

static uint32_t hiw(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return (uint32_t)(u >> 32);
}
static uint32_t low(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return (uint32_t)u;
}
static double sethi(double x, uint32_t h) {
    uint64_t u = ((uint64_t)h << 32) | low(x);
    double r;
    memcpy(&r, &u, 8);
    return r;
}

double or_det_log(double x) {
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                        two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                        Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                        Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k = 0, hx = (int32_t)hiw(x), i, j;
    uint32_t lx = low(x);
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -INFINITY;
        if (hx < 0) return NAN;
        k -= 54;
        x *= two54;
        hx = (int32_t)hiw(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    x = sethi(x, (uint32_t)(hx | (i ^ 0x3ff00000)));
    k += (i >> 20);
    f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0 + f);
    dk = (double)k;
    z = s * s;
    i = hx - 0x6147a;
    w = z * z;
    j = 0x6b851 - hx;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

double or_det_exp(double x) {
    static const double halF[2] = {0.5, -0.5}, o_threshold = 7.09782712893383973096e+02,
                        u_threshold = -7.45133219101941108420e+02,
                        ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01},
                        ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10},
                        invln2 = 1.44269504088896338700e+00, P1 = 1.66666666666666019037e-01,
                        P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
                        P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08,
                        twom1000 = 9.33263618503218878990e-302;
    double y, hi = 0.0, lo = 0.0, c, t;
    int32_t k = 0, xsb;
    uint32_t hx = hiw(x);
    xsb = (int32_t)((hx >> 31) & 1);
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | low(x)) != 0) return x + x;
            return xsb == 0 ? x : 0.0;
        }
        if (x > o_threshold) return INFINITY;
        if (x < u_threshold) return 0.0;
    }
    if (hx > 0x3fd62e42) {
        if (hx < 0x3FF0A2B2) {
            hi = x - ln2HI[xsb];
            lo = ln2LO[xsb];
            k = 1 - xsb - xsb;
        } else {
            k = (int32_t)(invln2 * x + halF[xsb]);
            t = k;
            hi = x - t * ln2HI[0];
            lo = t * ln2LO[0];
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {
        return 1.0 + x;
    } else
        k = 0;
    t = x * x;
    c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) return sethi(y, hiw(y) + ((uint32_t)k << 20));
    return sethi(y, hiw(y) + ((uint32_t)(k + 1000) << 20)) * twom1000;
}

/* FPC Math.power, non-integer exponent branch */
double or_fpc_power(double base, double exponent) {
    if (exponent == 0.0) return 1.0;
    if (base == 0.0 && exponent > 0.0) return 0.0;
    return or_det_exp(exponent * or_det_log(base));
}

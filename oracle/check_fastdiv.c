/* TEST INFRASTRUCTURE: exhaustive check that the GPU's fast x / 10000.0 (psyv.hip div10000<true>:
 * q0 = x * RN(1e-4), q = fma(fma(-q0, 1e4, x), RN(1e-4), q0)) equals the IEEE division for every colour
 * sum the gamma = -1 RGBToYUV (main.pas:2656-2679) can form: x = 2126 r/255 + 7152 g/255 + 722 b/255,
 * r, g, b in 0..255, evaluated left to right without contraction.  Prints the mismatch count. */
#include <math.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    const double inv = 1.0 / 10000.0;
    double lut[256];
    long bad = 0, tot = 0;
    for (int i = 0; i < 256; i++) lut[i] = i / 255.0;
    for (int r = 0; r < 256; r++)
        for (int g = 0; g < 256; g++)
            for (int b = 0; b < 256; b++) {
                volatile double a1 = 2126.0 * lut[r], a2 = 7152.0 * lut[g], a3 = 722.0 * lut[b];
                volatile double x = a1 + a2;
                x = x + a3;
                const double q = x / 10000.0;
                const double q0 = x * inv;
                const double q1 = fma(fma(-q0, 10000.0, x), inv, q0);
                tot++;
                if (memcmp(&q, &q1, sizeof q)) bad++;
            }
    printf("%ld %ld\n", tot, bad);
    return 0;
}

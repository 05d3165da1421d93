/*
 * load_kf.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the Load step's keyframe detection:
 *   btnLoadClick main.pas:1099-1146, ComputeInterFrameCorrelation main.pas:811-828,
 *   PearsonCorrelation main.pas:1465-1492, LoadFrame's FSPixels main.pas:3211-3264.
 *
 * FSPixels: LoadFrame writes FromRGB(SwapRB(bitmap pixel)) = r, g, b bytes of the tile pixel col
 * (0x00BBGGRR, the same value TilesRGBPixels holds) in screen raster order (main.pas:3248-3262),
 * then DitherFloydSteinberg(FSPixels) (main.pas:1966-1993).  With cBitsPerComp = 8 (main.pas:20)
 * Posterize(v) = min(255, (v*255 div 255)*(256 div 255)) = v (main.pas:703-709): every QuantError is 0
 * and the dither leaves the bytes unchanged, so FSPixels is read straight from the tiles here.
 *
 * Pearson: mean(x) = Sum / N (FPC Math; the sum of bytes is an exact integer in double), then ONE
 * sequential fp64 pass in array order (planar: all r, all g, all b), every op rounded, no FMA
 * (compiled -ffp-contract=off), sqrt / product / division as written.
 * Parity: no reference fixture exists for this path (no FPC, no frames in the reference): the
 * restatement is pinned by known-answer tests (tests/test_keyframes.py) -- "parity unpinned" against
 * the reference binary.
 */
#include <math.h>
#include <stdint.h>

#include "tiler_oracle.h"

/* frames: tile-major [tm_h*tm_w][64] int32 0x00BBGGRR (TFrame.Tiles[].RGBPixels, main.pas:3264-3266) */
static inline int fs_byte(const int32_t *f, int tm_w, int sy, int sx, int c) {
    const int32_t col = f[((long)(sy >> 3) * tm_w + (sx >> 3)) * 64 + (sy & 7) * 8 + (sx & 7)];
    return (col >> (8 * c)) & 0xff; /* FromRGB main.pas:578-583 */
}

double or_interframe_corr(const int32_t *a, const int32_t *b, int tm_w, int tm_h) {
    const int W = tm_w * 8, H = tm_h * 8;
    const long n = 3L * W * H;
    /* mean(x) main.pas:1472-1473: exact integer sums */
    uint64_t sa = 0, sb = 0;
    for (long t = 0; t < (long)tm_w * tm_h * 64; t++) {
        for (int c = 0; c < 3; c++) {
            sa += (a[t] >> (8 * c)) & 0xff;
            sb += (b[t] >> (8 * c)) & 0xff;
        }
    }
    const double mx = (double)sa / (double)n, my = (double)sb / (double)n;
    double num = 0.0, denx = 0.0, deny = 0.0;
    /* ya[i + sz*c] := FSPixels[i*3 + c] (main.pas:819-826): channel-major, raster inside */
    for (int c = 0; c < 3; c++)
        for (int sy = 0; sy < H; sy++)
            for (int sx = 0; sx < W; sx++) {
                const double x = (double)fs_byte(a, tm_w, sy, sx, c), y = (double)fs_byte(b, tm_w, sy, sx, c);
                const double dx = x - mx, dy = y - my;
                num += dx * dy; /* main.pas:1480 */
                denx += dx * dx; /* sqr(x[i] - mx) main.pas:1481 */
                deny += dy * dy;
            }
    denx = sqrt(denx);
    deny = sqrt(deny);
    const double den = denx * deny;
    double r = 0.0;
    if (den != 0.0) r = num / den;
    return r;
}

void or_interframe_corr_batch(const int32_t *frames, int F, int tm_w, int tm_h, double *corr) {
    const long fs = (long)tm_w * tm_h * 64;
    for (int i = 1; i < F; i++) corr[i - 1] = or_interframe_corr(frames + (i - 1) * fs, frames + i * fs, tm_w, tm_h);
}

/* btnLoadClick main.pas:1099-1146 (keyframe split).  corr[i-1] = ComputeInterFrameCorrelation(i-1, i).
 * kf_of_frame[F] := keyframe index of each frame; returns the keyframe count. */
int or_find_keyframes(const double *corr, int F, int tile_map_size, int32_t *kf_of_frame) {
    const int max_tiles_per_kf = 24 * 1920 * 1080 / 64; /* CShotTransMaxTilesPerKF main.pas:986 */
    const int grace = 24;                               /* CShotTransGracePeriod */
    const double savg = 6;                              /* CShotTransSAvgFrames */
    const double soft = 0.9, hard = 0.5;                /* CShotTransSoftThres / HardThres */
    if (F <= 0) return 0;
    int kf = 0, last = 0;
    double av = -1.0;
    kf_of_frame[0] = 0;
    for (int i = 1; i < F; i++) {
        const double v = corr[i - 1];
        if (av == -1.0)
            av = v;
        else
            av = av * (1.0 - 1.0 / savg) + v * (1.0 / savg);
        const double ratio = fmax(0.01, v) / fmax(0.01, av);
        const int is_kf = (ratio < hard) || ((ratio < soft) && ((i - last + 1) > grace)) ||
                          ((long)(i - last + 1) * tile_map_size > max_tiles_per_kf);
        if (is_kf) {
            kf++;
            av = -1.0;
            last = i;
        }
        kf_of_frame[i] = kf;
    }
    return kf + 1;
}

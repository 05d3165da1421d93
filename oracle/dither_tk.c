/*
 * dither_tk.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of FinishDitherTiles' per-tile work (the part after the palettes exist):
 *   DitherTile with Thomas Knoll mixing (the default: chkUseTK checked, main.lfm:272-282)  main.pas:1998-2055
 *   DeviseBestMixingPlanThomasKnoll                                                        main.pas:1828-1875
 *   PreparePlan (Y2Palette, LumaPal)                                                        main.pas:1494-1526
 *   ColorCompare                                                                            main.pas:1557-1571
 *   QuickSort (the reference's own, kmodes.pas:89-136) with PlanCompareLuma                  main.pas:1540-1551
 *   PrepareTileMirrors (canonical orientation)                                              main.pas:4049-4069
 * and the non-default branch (chkUseTK unchecked):
 *   DeviseBestMixingPlanYliluoma, the ASM_DBMP x86-64 form (main.pas:5 defines ASM_DBMP)    main.pas:1573-1826
 *   DitherTile's Yliluoma branch (map_value * count shr 6)                                  main.pas:2055-2067
 * The colour cache of the reference (CountCache / ListCache) only memoises the per-colour list: not restated.
 * Parity: no reference fixture exists (no FPC, no palettes in the reference): pinned by known-answer tests and an
 * independent Python restatement (tests/test_dither.py) -- "parity unpinned" against the binary.
 */
#include <stdint.h>
#include <string.h>

#include "tiler_oracle.h"

#define RED_MUL 2126
#define GREEN_MUL 7152
#define BLUE_MUL 722
#define LUMA_DIV (RED_MUL + GREEN_MUL + BLUE_MUL)
#define RGBW 13
#define DITHER_LEN 64

static const uint8_t k_dither_map[64] = { /* cDitheringMap main.pas:46-55 */
    0,  48, 12, 60, 3,  51, 15, 63, 32, 16, 44, 28, 35, 19, 47, 31, 8,  56, 4,  52, 11, 59,
    7,  55, 40, 24, 36, 20, 43, 27, 39, 23, 2,  50, 14, 62, 1,  49, 13, 61, 34, 18, 46, 30,
    33, 17, 45, 29, 10, 58, 6,  54, 9,  57, 5,  53, 42, 26, 38, 22, 41, 25, 37, 21};

const uint8_t *or_dither_map(void) { return k_dither_map; }

static int64_t color_compare(int64_t r1, int64_t g1, int64_t b1, int64_t r2, int64_t g2, int64_t b2) {
    const int64_t luma1 = r1 * RED_MUL + g1 * GREEN_MUL + b1 * BLUE_MUL;
    const int64_t luma2 = r2 * RED_MUL + g2 * GREEN_MUL + b2 * BLUE_MUL;
    const int64_t lumadiff = (luma1 - luma2) / LUMA_DIV; /* Pascal div: truncation toward zero, as C */
    const int64_t dr = r1 - r2, dg = g1 - g2, db = b1 - b2;
    int64_t r = (dr * dr) * RGBW;
    r += (dg * dg) * RGBW;
    r += (db * db) * RGBW;
    r += (lumadiff * lumadiff) << 5;
    return r;
}

static int cmp_luma(uint8_t a, uint8_t b, const int32_t *luma) { /* CompareValue(LumaPal[a], LumaPal[b]) */
    return luma[a] < luma[b] ? -1 : luma[a] > luma[b] ? 1 : 0;
}

/* kmodes.pas:89-136 on a byte array */
static void quicksort_bytes(uint8_t *a, int first, int last, const int32_t *luma) {
    if (last <= first) return;
    int i, j;
    do {
        i = first;
        j = last;
        int p = (first + last) >> 1;
        do {
            while (cmp_luma(a[i], a[p], luma) < 0) i++;
            while (cmp_luma(a[j], a[p], luma) > 0) j--;
            if (i <= j) {
                const uint8_t t = a[j];
                a[j] = a[i];
                a[i] = t;
                if (p == i)
                    p = j;
                else if (p == j)
                    p = i;
                i++;
                j--;
            }
        } while (i <= j);
        if (first < j) quicksort_bytes(a, first, j, luma);
        first = i;
    } while (i < last);
}

/* DeviseBestMixingPlanThomasKnoll main.pas:1828-1875: the sorted 64-entry list for colour col */
void or_tk_plan(const int32_t *pal, int palsize, int32_t col, uint8_t *list) {
    int32_t pr[256], pg[256], pb[256], luma[256];
    for (int i = 0; i < palsize; i++) { /* PreparePlan main.pas:1514-1525 */
        pr[i] = pal[i] & 0xff;
        pg[i] = (pal[i] >> 8) & 0xff;
        pb[i] = (pal[i] >> 16) & 0xff;
        luma[i] = pr[i] * RED_MUL + pg[i] * GREEN_MUL + pb[i] * BLUE_MUL;
    }
    const int64_t s[3] = {col & 0xff, (col >> 8) & 0xff, (col >> 16) & 0xff};
    int64_t e[3] = {0, 0, 0};
    for (int c = 0; c < DITHER_LEN; c++) {
        int64_t t[3];
        for (int k = 0; k < 3; k++) t[k] = s[k] + (e[k] * 9) / 100;
        int64_t least = INT64_MAX;
        int chosen = c & (palsize - 1);
        for (int idx = 0; idx < palsize; idx++) {
            const int64_t pen = color_compare(t[0], t[1], t[2], pr[idx], pg[idx], pb[idx]);
            if (pen < least) {
                least = pen;
                chosen = idx;
            }
        }
        list[c] = (uint8_t)chosen;
        e[0] += s[0];
        e[1] += s[1];
        e[2] += s[2];
        e[0] -= pr[chosen];
        e[1] -= pg[chosen];
        e[2] -= pb[chosen];
    }
    quicksort_bytes(list, 0, DITHER_LEN - 1, luma);
}

/* DeviseBestMixingPlanYliluoma main.pas:1573-1826 as the reference build runs it: main.pas:5 defines ASM_DBMP, so on
 * x86-64 the SSE block (1602-1752) replaces the Pascal loop.  Its arithmetic, lane by lane over (r, g, b, luma):
 * xmm4 = the colour (r, g, b, (r*cRedMul + g*cGreenMul + b*cBlueMul) div cLumaDiv), xmm5 = 1s, xmm6 = (13, 13, 13,
 * 32); per palette entry sum = so_far, add = Y2Palette[index] (r, g, b, LumaPal div cLumaDiv); per t sum += add and
 * add += 1 in all four lanes (the Pascal form leaves the luma lane alone), then
 * pen = sum_k w_k * (((gVecInv[t] * sum_k) shr 16) - x_k)^2, gVecInv[t] = 65536 div t, every product the low 32 bits
 * (pmulld), the shift logical (psrld), the four lanes added mod 2^32 (phaddd) and compared zero-extended, strict
 * '<' against the least so far (jae).  The chosen amount is t - plan_count, capped by the list (256 entries). */
#define YL_LIST 256
int or_yl_plan(const int32_t *pal, int palsize, int mixed, int32_t col, uint8_t *list) {
    uint32_t y2[256][4];
    int32_t luma[256];
    for (int i = 0; i < palsize; i++) { /* PreparePlan main.pas:1514-1525 */
        const uint32_t r = pal[i] & 0xff, g = (pal[i] >> 8) & 0xff, b = (pal[i] >> 16) & 0xff;
        luma[i] = (int32_t)(r * RED_MUL + g * GREEN_MUL + b * BLUE_MUL);
        y2[i][0] = r;
        y2[i][1] = g;
        y2[i][2] = b;
        y2[i][3] = (uint32_t)luma[i] / LUMA_DIV;
    }
    const uint32_t r = col & 0xff, g = (col >> 8) & 0xff, b = (col >> 16) & 0xff;
    const uint32_t x[4] = {r, g, b, (r * RED_MUL + g * GREEN_MUL + b * BLUE_MUL) / LUMA_DIV};
    const uint32_t w[4] = {RGBW, RGBW, RGBW, 32};
    uint32_t so_far[4] = {0, 0, 0, 0};
    int plan_count = 0;
    while (plan_count < mixed) {
        const int max_test = plan_count == 0 ? 1 : plan_count;
        uint64_t least = 0x7fffffffffffffffull;
        int chosen = 0, chosen_t = plan_count + 1;
        for (int idx = 0; idx < palsize; idx++) {
            uint32_t sum[4], add[4];
            for (int k = 0; k < 4; k++) {
                sum[k] = so_far[k];
                add[k] = y2[idx][k];
            }
            for (int t = plan_count + 1; t <= plan_count + max_test; t++) {
                const uint32_t inv = 65536u / (uint32_t)t;
                uint32_t pen = 0;
                for (int k = 0; k < 4; k++) {
                    sum[k] += add[k];
                    add[k] += 1u;
                    const uint32_t q = (inv * sum[k]) >> 16;
                    const uint32_t d = q - x[k];
                    pen += (d * d) * w[k];
                }
                if ((uint64_t)pen < least) {
                    least = pen;
                    chosen = idx;
                    chosen_t = t;
                }
            }
        }
        int amount = chosen_t - plan_count;
        if (amount > YL_LIST - plan_count) amount = YL_LIST - plan_count;
        memset(list + plan_count, chosen, (size_t)amount);
        plan_count += amount;
        for (int k = 0; k < 4; k++) so_far[k] += y2[chosen][k] * (uint32_t)amount;
    }
    quicksort_bytes(list, 0, plan_count - 1, luma);
    return plan_count;
}

/* FinishDitherTiles' per-tile work (main.pas:2507-2524): DitherTile (Thomas Knoll) with the tile's
 * DitheringPalIndex palette, then PrepareTileMirrors.  rgb[n][64] 0x00BBGGRR, pal_of[n], palettes[P][palsize]. */
static void dither_tiles(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int palsize,
                         int yl_mixed, uint8_t *palpix, uint8_t *hm, uint8_t *vm) {
    uint8_t list[YL_LIST];
    for (int i = 0; i < n; i++) {
        const int32_t *pal = palettes + (long)pal_of[i] * palsize;
        uint8_t px[64];
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                if (yl_mixed > 0) { /* DitherTile's Yliluoma branch main.pas:2057-2066 */
                    const int count = or_yl_plan(pal, palsize, yl_mixed, rgb[(long)i * 64 + y * 8 + x], list);
                    px[y * 8 + x] = list[(k_dither_map[y * 8 + x] * count) >> 6];
                } else {
                    or_tk_plan(pal, palsize, rgb[(long)i * 64 + y * 8 + x], list);
                    px[y * 8 + x] = list[k_dither_map[y * 8 + x]];
                }
            }
        /* PrepareTileMirrors: quadrant sums, v outer / h inner, strict '>' (first max) */
        int best = -1, bh = 0, bv = 0;
        for (int vf = 0; vf < 2; vf++)
            for (int hf = 0; hf < 2; hf++) {
                int v = 0;
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) v += px[(y + 4 * vf) * 8 + x + 4 * hf];
                if (v > best) {
                    best = v;
                    bh = hf;
                    bv = vf;
                }
            }
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                palpix[(long)i * 64 + y * 8 + x] = px[(bv ? 7 - y : y) * 8 + (bh ? 7 - x : x)];
        hm[i] = (uint8_t)bh;
        vm[i] = (uint8_t)bv;
    }
}

void or_dither_tiles_tk(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int palsize,
                        uint8_t *palpix, uint8_t *hm, uint8_t *vm) {
    dither_tiles(n, rgb, pal_of, palettes, palsize, 0, palpix, hm, vm);
}

void or_dither_tiles_yl(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int palsize,
                        int mixed, uint8_t *palpix, uint8_t *hm, uint8_t *vm) {
    dither_tiles(n, rgb, pal_of, palettes, palsize, mixed, palpix, hm, vm);
}

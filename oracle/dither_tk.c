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

/* FinishDitherTiles' per-tile work (main.pas:2507-2524): DitherTile (Thomas Knoll) with the tile's
 * DitheringPalIndex palette, then PrepareTileMirrors.  rgb[n][64] 0x00BBGGRR, pal_of[n], palettes[P][palsize]. */
void or_dither_tiles_tk(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int palsize,
                        uint8_t *palpix, uint8_t *hm, uint8_t *vm) {
    uint8_t list[DITHER_LEN];
    for (int i = 0; i < n; i++) {
        const int32_t *pal = palettes + (long)pal_of[i] * palsize;
        uint8_t px[64];
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                or_tk_plan(pal, palsize, rgb[(long)i * 64 + y * 8 + x], list);
                px[y * 8 + x] = list[k_dither_map[y * 8 + x]];
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

/*
 * palette.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the palette-generation half of the Dither step, default settings
 * (chkUseDL3 checked, cbxDLBPC 7: main.lfm:262-268, 502):
 *   QuantizePalette with DoDennisLeeV3                                  main.pas:2154-2254, 2396-2433
 *     dl3quant: build_table3 / setrgb / calc_err / recount_next /       dlquant/quantizer.c:437-663
 *               recount_dist / reduce_table3 / set_palette3
 *     CMPal.Sort(CompareCMULHS) (TFPList.Sort)                          main.pas:2081-2090, 2413
 *     FColorMap HSV bytes (RGBToHSV, Windows MulDiv) and luma            main.pas:3496-3543, 4835-4847
 *   FinishQuantizePalette: palettes by UseCount (kmodes.pas QuickSort)   main.pas:2435-2480, kmodes.pas:89-136
 *
 * Integer widths follow the reference DLL's target (dlquant_dll.vcxproj, MSVC, LLP64): quantizer.h's `ulong` is
 * 32 bits, so CUBE3's colour sums and counts wrap modulo 2^32 exactly as there.  calc_err is the float function of
 * quantizer.c:512-541 (its forward declaration at :357 says ulong; every caller stores the value into a float).
 *
 * Parity: quantizer.c cannot be compiled here without stand-ins (MSVC-only __declspec/__stdcall in quantizer.h,
 * the progress_init/progress_update/progress_end callbacks it calls are defined elsewhere in mtPaint, and the two
 * calc_err declarations conflict), and the reference holds no DLv3 fixture: this restatement is "parity unpinned"
 * against the binary.  TFPList.Sort's tie order (only for distinct colours with equal luma, V, S and H) follows the
 * classic FPC RTL QuickSort (lists.inc); the RTL source is not in the reference -- also unpinned.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tiler_oracle.h"

/* ------------------------------------------------------------------------------------------------------------
 * dl3quant (quantizer.c:437-663)
 * ------------------------------------------------------------------------------------------------------------ */
typedef struct {
    uint32_t r, g, b, pixel_count; /* ulong (32-bit) */
    float err;
    int32_t cc;
    uint8_t rr, gg, bb;
} cube3;

typedef struct {
    cube3 *t;
    int tot_colors;
    float sqr_tbl[511]; /* init_table, quantizer.c:457-470 */
} dl3ctx;

static float sq3(const dl3ctx *c, int d) { return c->sqr_tbl[d + 255]; }

static void setrgb(cube3 *rec) { /* quantizer.c:472-478 */
    const int v = (int)rec->pixel_count, v2 = v >> 1;
    rec->rr = (uint8_t)((rec->r + (uint32_t)v2) / (uint32_t)v);
    rec->gg = (uint8_t)((rec->g + (uint32_t)v2) / (uint32_t)v);
    rec->bb = (uint8_t)((rec->b + (uint32_t)v2) / (uint32_t)v);
}

static float calc_err(const dl3ctx *c, int c1, int c2) { /* quantizer.c:512-541 */
    const cube3 *a = c->t + c1, *b = c->t + c2;
    const uint32_t P1 = a->pixel_count, P2 = b->pixel_count, P3 = P1 + P2;
    const int R3 = (int)((a->r + b->r + (P3 >> 1)) / P3);
    const int G3 = (int)((a->g + b->g + (P3 >> 1)) / P3);
    const int B3 = (int)((a->b + b->b + (P3 >> 1)) / P3);
    const int R1 = a->rr, G1 = a->gg, B1 = a->bb, R2 = b->rr, G2 = b->gg, B2 = b->bb;
    float dist1 = sq3(c, R3 - R1) + sq3(c, G3 - G1) + sq3(c, B3 - B1);
    dist1 = sqrtf(dist1) * (float)P1;
    float dist2 = sq3(c, R2 - R3) + sq3(c, G2 - G3) + sq3(c, B2 - B3);
    dist2 = sqrtf(dist2) * (float)P2;
    return dist1 + dist2;
}

static void recount_next(dl3ctx *c, int i) { /* quantizer.c:543-560 */
    int c2 = 0;
    float err = HUGE_VALF;
    for (int j = i + 1; j < c->tot_colors; j++) {
        const float cur = calc_err(c, i, j);
        if (cur < err) {
            err = cur;
            c2 = j;
        }
    }
    c->t[i].err = err;
    c->t[i].cc = c2;
}

static void recount_dist(dl3ctx *c, int c1) { /* quantizer.c:562-581 */
    recount_next(c, c1);
    for (int i = 0; i < c1; i++) {
        if (c->t[i].cc == c1)
            recount_next(c, i);
        else {
            const float cur = calc_err(c, i, c1);
            if (cur < c->t[i].err) {
                c->t[i].err = cur;
                c->t[i].cc = c1;
            }
        }
    }
}

static void reduce_table3(dl3ctx *c, int num_colors) { /* quantizer.c:583-648 (no progress bail-out) */
    int i, c1 = 0, c2 = 0;
    for (i = 0; i < c->tot_colors - 1; i++) recount_next(c, i);
    if (c->tot_colors > 0) { /* i = max(0, tot_colors - 1): the reference writes entry 0 of an empty table too */
        c->t[i].err = HUGE_VALF;
        c->t[i].cc = c->tot_colors;
    }
    while (c->tot_colors > num_colors) {
        float err = HUGE_VALF;
        for (i = 0; i < c->tot_colors; i++)
            if (c->t[i].err < err) {
                err = c->t[i].err;
                c1 = i;
            }
        c2 = c->t[c1].cc;
        c->t[c2].r += c->t[c1].r;
        c->t[c2].g += c->t[c1].g;
        c->t[c2].b += c->t[c1].b;
        c->t[c2].pixel_count += c->t[c1].pixel_count;
        setrgb(c->t + c2);
        c->tot_colors--;
        c->t[c1] = c->t[c->tot_colors];
        c->t[c->tot_colors - 1].err = HUGE_VALF;
        c->t[c->tot_colors - 1].cc = c->tot_colors;
        for (i = 0; i < c1; i++)
            if (c->t[i].cc == c->tot_colors) c->t[i].cc = c1;
        for (i = c1 + 1; i < c->tot_colors; i++)
            if (c->t[i].cc == c->tot_colors) recount_next(c, i);
        recount_dist(c, c1);
        if (c2 != c->tot_colors) recount_dist(c, c2);
    }
}

/* dl3quant(inbuf, width * height = npix, quant_to, lookup_bpc, userpal): the first quant_to palette entries as
 * pal[i] = r | g << 8 | b << 16 (0 past the table, the reference's calloc'd context).  Returns the colour count
 * of the histogram (tot_colors before reduction). */
int or_dl3quant(const uint8_t *rgb, long npix, int quant_to, int lookup_bpc, int32_t *pal) {
    const long lookup_size = 1L << (lookup_bpc * 3);
    dl3ctx *c = (dl3ctx *)calloc(1, sizeof(dl3ctx));
    c->t = (cube3 *)calloc((size_t)lookup_size, sizeof(cube3));
    for (int i = -255; i <= 255; i++) c->sqr_tbl[i + 255] = (float)(i * i);
    const int mbpc = (1 << lookup_bpc) - 1;
    for (long i = 0; i < npix; i++) { /* build_table3, quantizer.c:480-510 */
        const uint8_t *im = rgb + 3 * i;
        const int r = im[0] * mbpc / 255, g = im[1] * mbpc / 255, b = im[2] * mbpc / 255;
        const long index = b | (g << lookup_bpc) | (r << (lookup_bpc << 1));
        c->t[index].r += im[0];
        c->t[index].g += im[1];
        c->t[index].b += im[2];
        c->t[index].pixel_count++;
    }
    c->tot_colors = 0;
    for (long i = 0; i < lookup_size; i++)
        if (c->t[i].pixel_count) {
            setrgb(c->t + i);
            c->t[c->tot_colors++] = c->t[i];
        }
    const int hist = c->tot_colors;
    reduce_table3(c, quant_to);
    for (int i = 0; i < quant_to; i++) /* set_palette3 + copy_pal */
        pal[i] = i < c->tot_colors ? (int32_t)(c->t[i].rr | (c->t[i].gg << 8) | (c->t[i].bb << 16)) : 0;
    free(c->t);
    free(c);
    return hist;
}

/* ------------------------------------------------------------------------------------------------------------
 * FColorMap (main.pas:4835-4847, cRGBBitsPerComp = 8: the identity colour map) and RGBToHSV (main.pas:3496-3543)
 * ------------------------------------------------------------------------------------------------------------ */
static int win_muldiv(int a, int b, int c) { /* Windows MulDiv: 64-bit product, rounded half away from zero */
    if (c == 0) return -1;
    if (c < 0) {
        a = -a;
        c = -c;
    }
    int64_t r;
    if ((a < 0 && b < 0) || (a >= 0 && b >= 0))
        r = ((int64_t)a * b + c / 2) / c;
    else
        r = ((int64_t)a * b - c / 2) / c;
    if (r > 2147483647LL || r < -2147483647LL) return -1;
    return (int)r;
}

void or_rgb_to_hsv(int32_t col, uint8_t *h, uint8_t *s, uint8_t *v) {
    const int rr = col & 0xff, gg = (col >> 8) & 0xff, bb = (col >> 16) & 0xff;
    int mx = rr, mn = rr;
    if (mx < gg) mx = gg;
    if (mx < bb) mx = bb;
    if (mn > gg) mn = gg;
    if (mn > bb) mn = bb;
    int hh = 0, ss = 0;
    const int ll = mx;
    if (ll != mn) {
        const int delta = ll - mn;
        ss = win_muldiv(delta, 255, ll);
        if (rr == ll)
            hh = win_muldiv(42, gg - bb, delta);
        else if (gg == ll)
            hh = win_muldiv(42, bb - rr, delta) + 84;
        else if (bb == ll)
            hh = win_muldiv(42, rr - gg, delta) + 168;
        hh = hh % 252; /* Pascal mod: sign of the dividend, as C */
    }
    *h = (uint8_t)(hh & 0xff);
    *s = (uint8_t)(ss & 0xff);
    *v = (uint8_t)(ll & 0xff);
}

int32_t or_color_luma(int32_t col) {
    return ((col & 0xff) * 2126 + ((col >> 8) & 0xff) * 7152 + ((col >> 16) & 0xff) * 722) / 10000;
}

/* ------------------------------------------------------------------------------------------------------------
 * CMPal.Sort(@CompareCMULHS): TFPList.Sort = the classic FPC RTL QuickSort on the pointer list
 * ------------------------------------------------------------------------------------------------------------ */
typedef struct {
    int32_t count, index, luma; /* TCountIndexArray, main.pas:193-196 */
    uint8_t hue, sat, val, dummy;
} count_index;

static int cmp_value(int a, int b) { return a < b ? -1 : a > b ? 1 : 0; }

static int compare_cmulhs(const count_index *a, const count_index *b) { /* main.pas:2081-2090 */
    int r = cmp_value(a->luma, b->luma);
    if (r == 0) r = cmp_value(a->val, b->val);
    if (r == 0) r = cmp_value(a->sat, b->sat);
    if (r == 0) r = cmp_value(a->hue, b->hue);
    return r;
}

static void fpc_list_quicksort(const count_index **l, int L, int R) {
    int I, J;
    do {
        I = L;
        J = R;
        const count_index *P = l[(L + R) / 2];
        do {
            while (compare_cmulhs(P, l[I]) > 0) I++;
            while (compare_cmulhs(P, l[J]) < 0) J--;
            if (I <= J) {
                const count_index *q = l[I];
                l[I] = l[J];
                l[J] = q;
                I++;
                J--;
            }
        } while (I <= J);
        if (L < J) fpc_list_quicksort(l, L, J);
        L = I;
    } while (I < R);
}

/* the tile palette of DoDennisLeeV3's colours: CMUsage items (main.pas:2239-2250) sorted (main.pas:2413-2417) */
void or_sort_cmulhs(const int32_t *cols, int n, int32_t *out) {
    count_index *items = (count_index *)calloc((size_t)n, sizeof(count_index));
    const count_index **l = (const count_index **)calloc((size_t)n, sizeof(void *));
    for (int i = 0; i < n; i++) {
        items[i].index = cols[i];
        items[i].count = 1;
        or_rgb_to_hsv(cols[i], &items[i].hue, &items[i].sat, &items[i].val);
        items[i].luma = or_color_luma(cols[i]);
        l[i] = items + i;
    }
    if (n > 1) fpc_list_quicksort(l, 0, n - 1);
    for (int i = 0; i < n; i++) out[i] = l[i]->index;
    free(l);
    free(items);
}

/* ------------------------------------------------------------------------------------------------------------
 * QuantizePalette, all palettes of one keyframe (main.pas:2154-2254, 2396-2433; the keyframe's tiles in frame
 * order are rgb[n][64] 0x00BBGGRR, their DitheringPalIndex pal_of[n], Active active[n] (null: all)).
 * pal_out[P][palsize] = PaletteIndexes, use_count[P] = PaletteUseCount.UseCount; hist[P] = DLv3 colour counts.
 * ------------------------------------------------------------------------------------------------------------ */
typedef struct {
    const int32_t *rgb, *pal_of;
    const uint8_t *active;
    long n;
    int P, palsize, bpc;
    int32_t *pal_out, *use_count, *hist;
} quant_job;

static void quantize_one(const quant_job *j, long p) {
    long cnt = 0;
    for (long t = 0; t < j->n; t++)
        if ((!j->active || j->active[t]) && j->pal_of[t] == p) cnt++;
    uint8_t *px = (uint8_t *)malloc((size_t)(cnt > 0 ? cnt : 1) * 64 * 3);
    long k = 0;
    for (long t = 0; t < j->n; t++) /* the tile rectangle's pixel order does not change the histogram */
        if ((!j->active || j->active[t]) && j->pal_of[t] == p)
            for (int x = 0; x < 64; x++, k++) {
                const int32_t c = j->rgb[t * 64 + x];
                px[3 * k] = (uint8_t)(c & 0xff);
                px[3 * k + 1] = (uint8_t)((c >> 8) & 0xff);
                px[3 * k + 2] = (uint8_t)((c >> 16) & 0xff);
            }
    int32_t *cols = (int32_t *)malloc((size_t)j->palsize * sizeof(int32_t));
    const int h = or_dl3quant(px, cnt * 64, j->palsize, j->bpc, cols);
    or_sort_cmulhs(cols, j->palsize, j->pal_out + p * j->palsize);
    j->use_count[p] = (int32_t)cnt;
    if (j->hist) j->hist[p] = h;
    free(cols);
    free(px);
}

typedef struct {
    quant_job *job;
    int P;
    int next;
    pthread_mutex_t mu;
} quant_pool;

static void *quant_worker(void *arg) { /* palettes are independent (DoQuantize per palette, main.pas:872-875) */
    quant_pool *q = (quant_pool *)arg;
    for (;;) {
        pthread_mutex_lock(&q->mu);
        const int p = q->next++;
        pthread_mutex_unlock(&q->mu);
        if (p >= q->P) return NULL;
        quantize_one(q->job, p);
    }
}

void or_quantize_palettes(const int32_t *rgb, const int32_t *pal_of, const uint8_t *active, long n, int P,
                          int palsize, int bpc, int32_t *pal_out, int32_t *use_count, int32_t *hist, int threads) {
    quant_job j = {rgb, pal_of, active, n, P, palsize, bpc, pal_out, use_count, hist};
    quant_pool q = {&j, P, 0, PTHREAD_MUTEX_INITIALIZER};
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    pthread_t th[64];
    for (int i = 1; i < threads; i++) pthread_create(&th[i], NULL, quant_worker, &q);
    quant_worker(&q);
    for (int i = 1; i < threads; i++) pthread_join(th[i], NULL);
}

/* ------------------------------------------------------------------------------------------------------------
 * FinishQuantizePalette (main.pas:2435-2480): the reference QuickSort (kmodes.pas:89-136) of the PaletteUseCount
 * records with ComparePaletteUseCount (use count descending, main.pas:2092-2095); lut[old] = new position.
 * ------------------------------------------------------------------------------------------------------------ */
typedef struct {
    int32_t use_count, pal_idx;
} pal_use;

static int cmp_pal_use(const pal_use *a, const pal_use *b) { return cmp_value(b->use_count, a->use_count); }

static void km_quicksort_paluse(pal_use *a, int first, int last) {
    if (last <= first) return;
    int i, j;
    do {
        i = first;
        j = last;
        int p = (first + last) >> 1;
        do {
            while (cmp_pal_use(a + i, a + p) < 0) i++;
            while (cmp_pal_use(a + j, a + p) > 0) j--;
            if (i <= j) {
                const pal_use t = a[j];
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
        if (first < j) km_quicksort_paluse(a, first, j);
        first = i;
    } while (i < last);
}

void or_finish_quantize_order(const int32_t *use_count, int P, int32_t *lut) {
    pal_use *a = (pal_use *)malloc((size_t)P * sizeof(pal_use));
    for (int p = 0; p < P; p++) {
        a[p].use_count = use_count[p];
        a[p].pal_idx = p;
    }
    km_quicksort_paluse(a, 0, P - 1);
    for (int p = 0; p < P; p++) lut[a[p].pal_idx] = p;
    free(a);
}

/*
 * tiler_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference hot path.
 * See tiler_oracle.h for the contract.  Compiled with -O2 -ffp-contract=off (oracle/Makefile).
 * Reference = /root/reference (b0nefish/tiler, FreePascal); citations are file:line there.
 */
#include "tiler_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>


/* ------------------------------------------------------------------------------------------
 * LUTs: InitLuts main.pas:592-642 (gamma 601-606, DCT 615-623).  gGamma main.pas:586.
 * ---------------------------------------------------------------------------------------- */
static double g_gamma[2] = {2.0, 0.6};
static double g_gamma_lut[3][256];
static double g_dct_lut[4096];
static int g_init = 0;

static void build_luts(void) {
    for (int g = -1; g <= 1; g++)
        for (int i = 0; i < 256; i++)
            g_gamma_lut[g + 1][i] = (g >= 0) ? pow(i / 255.0, g_gamma[g]) : i / 255.0;
    int i = 0;
    for (int v = 0; v < 8; v++)
        for (int u = 0; u < 8; u++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    /* cos((x + 0.5) * u * PI / 16.0) * cos((y + 0.5) * v * PI / 16.0) */
                    double a = (((double)x + 0.5) * (double)u) * M_PI / 16.0;
                    double b = (((double)y + 0.5) * (double)v) * M_PI / 16.0;
                    g_dct_lut[i++] = cos(a) * cos(b);
                }
    g_init = 1;
}

void or_init(void) {
    if (!g_init) build_luts();
}
void or_set_gamma(double g0, double g1) {
    g_gamma[0] = g0;
    g_gamma[1] = g1;
    build_luts();
}
const double *or_dct_lut(void) {
    or_init();
    return g_dct_lut;
}
const double *or_gamma_lut(void) {
    or_init();
    return &g_gamma_lut[0][0];
}

/* cDCTQuantization main.pas:63-98 (cQ = sqrt(16) = 4) as the q denominators. */
static const int k_qden[3][64] = {
    {16, 11, 10, 16, 24, 40, 51, 61,   12, 12, 14, 19, 26, 58, 60, 55,   14, 13, 16, 24, 40, 57, 69, 56,
     14, 17, 22, 29, 51, 87, 80, 62,   18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99},
    {17, 18, 24, 47, 99, 99, 99, 99,   18, 21, 26, 66, 99, 99, 99, 112,  24, 26, 56, 99, 99, 99, 112, 128,
     47, 66, 99, 99, 99, 112, 128, 144, 99, 99, 99, 99, 112, 128, 144, 160, 99, 99, 99, 112, 128, 144, 160, 176,
     99, 99, 112, 128, 144, 160, 176, 192, 99, 112, 128, 144, 160, 176, 192, 208},
    {17, 18, 24, 47, 99, 99, 99, 99,   18, 21, 26, 66, 99, 99, 99, 112,  24, 26, 56, 99, 99, 99, 112, 128,
     47, 66, 99, 99, 99, 112, 128, 144, 99, 99, 99, 99, 112, 128, 144, 160, 99, 99, 99, 112, 128, 144, 160, 176,
     99, 99, 112, 128, 144, 160, 176, 192, 99, 112, 128, 144, 160, 176, 192, 208}};

/* RGBToYUV main.pas:2656-2679 (cRedMul/cGreenMul/cBlueMul main.pas:26-28). */
static inline void rgb_to_yuv(int32_t col, int gamma, double *y, double *u, double *v) {
    int r = col & 0xff, g = (col >> 8) & 0xff, b = (col >> 16) & 0xff;
    double fr, fg, fb;
    if (gamma >= 0) {
        fr = g_gamma_lut[gamma + 1][r];
        fg = g_gamma_lut[gamma + 1][g];
        fb = g_gamma_lut[gamma + 1][b];
    } else {
        fr = r / 255.0;
        fg = g / 255.0;
        fb = b / 255.0;
    }
    double yy = (2126.0 * fr + 7152.0 * fg + 722.0 * fb) / 10000.0;
    double uu = (fb - yy) * (0.5 / (1.0 - 722.0 / 10000.0));
    double vv = (fr - yy) * (0.5 / (1.0 - 2126.0 / 10000.0));
    *y = yy;
    *u = uu;
    *v = vv;
}

/* RGBToLAB main.pas:2711-2747 (D50, Wright-Guild XYZ) with FPC Math.power = exp(e * ln(b)) (detmath.c). */
static inline void rgb_to_lab(int32_t col, int gamma, double *ol, double *oa, double *ob) {
    const int ir = col & 0xff, ig = (col >> 8) & 0xff, ib = (col >> 16) & 0xff;
    double c[3];
    const int ch[3] = {ir, ig, ib};
    for (int k = 0; k < 3; k++) {
        double v = gamma >= 0 ? g_gamma_lut[gamma + 1][ch[k]] : ch[k] / 255.0; /* GammaCorrect */
        if (v > 0.04045)
            v = or_fpc_power((v + 0.055) / 1.055, 2.4);
        else
            v = v / 12.92;
        c[k] = v;
    }
    const double r = c[0], g = c[1], b = c[2];
    double x = (r * 0.49000 + g * 0.31000 + b * 0.20000) / 0.17697;
    double y = (r * 0.17697 + g * 0.81240 + b * 0.01063) / 0.17697;
    double z = (r * 0.00000 + g * 0.01000 + b * 0.99000) / 0.17697;
    x /= 96.6797 / 100;
    y /= 100.000 / 100;
    z /= 82.5188 / 100;
    if (x > 0.008856) x = or_fpc_power(x, 1.0 / 3.0); else x = (7.787 * x) + 16.0 / 116.0;
    if (y > 0.008856) y = or_fpc_power(y, 1.0 / 3.0); else y = (7.787 * y) + 16.0 / 116.0;
    if (z > 0.008856) z = or_fpc_power(z, 1.0 / 3.0); else z = (7.787 * z) + 16.0 / 116.0;
    *ol = (116 * y) - 16;
    *oa = 500 * (x - y);
    *ob = 200 * (y - z);
}

/* WaveletGS main.pas:2805-2840 (normalized Haar, recursion on the top-left quadrant). */
static void wavelet_gs(const double *data, double *output, int dx, int dy, int depth) {
    double tx[64], ty[64];
    memset(tx, 0, sizeof(tx));
    memset(ty, 0, sizeof(ty));
    const double factor = 1.0 / sqrt(2.0);
    for (int y = 0; y < dy; y++) {
        int off = y * 8;
        for (int x = 0; x < dx / 2; x++) {
            tx[x + off] = (data[x * 2 + off] + data[x * 2 + 1 + off]) * factor;
            tx[x + dx / 2 + off] = (data[x * 2 + off] - data[x * 2 + 1 + off]) * factor;
        }
    }
    for (int x = 0; x < dx; x++)
        for (int y = 0; y < dy / 2; y++) {
            ty[x + y * 8] = (tx[x + y * 2 * 8] + tx[x + (y * 2 + 1) * 8]) * factor;
            ty[x + (y + dy / 2) * 8] = (tx[x + y * 2 * 8] - tx[x + (y * 2 + 1) * 8]) * factor;
        }
    for (int y = 0; y < dy; y++) memcpy(&output[y * 8], &ty[y * 8], (size_t)dx * sizeof(double));
    if (depth > 0) wavelet_gs(output, output, dx / 2, dy / 2, depth - 1);
}

/* ComputeTilePsyVisFeatures main.pas:2997-3177 (UseLAB only for the Dither step's descriptors, OR_LAB). */
void or_psyv(const int32_t *rgb, const uint8_t *palpix, const int32_t *pal, int flags, int gamma, double *out) {
    or_init();
    double cpn[3][64];
    const int hm = (flags & OR_HMIRROR) != 0, vm = (flags & OR_VMIRROR) != 0;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            int xx = hm ? 7 - x : x;
            int yy = vm ? 7 - y : y;
            int32_t col = (flags & OR_FROM_PAL) ? pal[palpix[yy * 8 + xx]] : rgb[yy * 8 + xx];
            if (flags & OR_LAB)
                rgb_to_lab(col, gamma, &cpn[0][y * 8 + x], &cpn[1][y * 8 + x], &cpn[2][y * 8 + x]);
            else
                rgb_to_yuv(col, gamma, &cpn[0][y * 8 + x], &cpn[1][y * 8 + x], &cpn[2][y * 8 + x]);
        }
    if (flags & OR_WAVELETS) {
        for (int c = 0; c < 3; c++) wavelet_gs(cpn[c], out + c * 64, 8, 8, 2);
    } else {
        const double sh = sqrt(0.5);
        for (int c = 0; c < 3; c++) {
            const double *lut = g_dct_lut;
            for (int v = 0; v < 8; v++)
                for (int u = 0; u < 8; u++) {
                    double z = 0.0;
                    for (int k = 0; k < 64; k++) z += cpn[c][k] * *lut++;
                    if (flags & OR_QWEIGHT) z *= 4.0 / sqrt((double)k_qden[c][v * 8 + u]);
                    double ratio = (u == 0 && v == 0) ? 0.5 : ((u == 0 || v == 0) ? sh : 1.0); /* cUVRatio 3000-3009 */
                    out[c * 64 + v * 8 + u] = z * ratio;
                }
        }
    }
}

void or_psyv_batch(int n, const int32_t *rgb, const uint8_t *palpix, const int32_t *pals, const int32_t *pal_of,
                   const uint8_t *flags_per, int flags, int gamma, double *out) {
    for (int i = 0; i < n; i++) {
        int f = flags | (flags_per ? flags_per[i] : 0);
        const int32_t *pal = (f & OR_FROM_PAL) ? pals + 16 * (pal_of ? pal_of[i] : 0) : NULL;
        or_psyv(rgb ? rgb + 64 * (size_t)i : NULL, palpix ? palpix + 64 * (size_t)i : NULL, pal, f, gamma,
                out + 192 * (size_t)i);
    }
}

/* ------------------------------------------------------------------------------------------
 * ANN 1.1.2 exact search semantics (from ANN.dll leaf scan RVA ~0x126d0):
 * dist accumulates t*t in fp32 with every op rounded; ties keep the first found.  The
 * canonical order here is candidate index order (ANN's kd-tree order: parity unpinned).
 * ---------------------------------------------------------------------------------------- */
float or_dist(const float *a, const float *b, int d) {
    float dist = 0.0f;
    for (int i = 0; i < d; i++) {
        float t = a[i] - b[i];
        float s = t * t;
        dist = dist + s;
    }
    return dist;
}

/* leaf-scan form with ANN's early break (dist > min_dist): same argmin, faster. */
static inline int nn_scan(const float *data, int n, int d, const float *q, float *err) {
    float best = FLT_MAX;
    int bi = -1;
    for (int j = 0; j < n; j++) {
        const float *p = data + (size_t)j * d;
        float dist = 0.0f;
        int i;
        for (i = 0; i < d; i++) {
            float t = q[i] - p[i];
            float s = t * t;
            dist = dist + s;
            if (dist > best) break;
        }
        if (i >= d && (bi < 0 || dist < best)) {
            best = dist;
            bi = j;
        }
    }
    if (err) *err = best;
    return bi;
}

int or_nn(const float *data, int n, int d, const float *q, float *err) { return nn_scan(data, n, d, q, err); }

/* annkSearch k-list (ANNmin_k::insert): shift only entries with key > dist -> equal keys keep
 * first found; results ascending.  Missing entries: idx -1, err FLT_MAX. */
void or_knn(const float *data, int n, int d, const float *q, int k, int *idx, float *err) {
    for (int i = 0; i < k; i++) {
        idx[i] = -1;
        err[i] = FLT_MAX;
    }
    int cnt = 0;
    for (int j = 0; j < n; j++) {
        float dist = or_dist(q, data + (size_t)j * d, d);
        float maxk = (cnt < k) ? FLT_MAX : err[k - 1];
        if (cnt == k && dist > maxk) continue;
        if (cnt == k && dist == maxk) continue; /* goes to slot k, dropped */
        int i = (cnt < k) ? cnt : k - 1;
        while (i > 0 && err[i - 1] > dist) {
            err[i] = err[i - 1];
            idx[i] = idx[i - 1];
            i--;
        }
        err[i] = dist;
        idx[i] = j;
        if (cnt < k) cnt++;
    }
}

typedef struct {
    const float *data, *q;
    int n, d, nq, t, threads;
    int *idx;
    float *err;
} nn_job;

static void *nn_worker(void *p) {
    nn_job *j = (nn_job *)p;
    for (int i = j->t; i < j->nq; i += j->threads)
        j->idx[i] = nn_scan(j->data, j->n, j->d, j->q + (size_t)i * j->d, &j->err[i]);
    return NULL;
}

void or_nn_batch(const float *data, int n, int d, const float *q, int nq, int *idx, float *err, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    nn_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (nn_job){data, q, n, d, nq, t, threads, idx, err};
        pthread_create(&th[t], NULL, nn_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------------------------
 * FrameTiling preparation.
 * ---------------------------------------------------------------------------------------- */

/* HMirrorPalTile / VMirrorPalTile main.pas:3179-3209 */
static void hflip(uint8_t *t) {
    for (int j = 0; j < 8; j++)
        for (int i = 0; i < 4; i++) {
            uint8_t v = t[j * 8 + i];
            t[j * 8 + i] = t[j * 8 + 7 - i];
            t[j * 8 + 7 - i] = v;
        }
}
static void vflip(uint8_t *t) {
    for (int j = 0; j < 4; j++)
        for (int i = 0; i < 8; i++) {
            uint8_t v = t[j * 8 + i];
            t[j * 8 + i] = t[(7 - j) * 8 + i];
            t[(7 - j) * 8 + i] = v;
        }
}

/* PrepareGlobalFT main.pas:3736-3780: per active tile, rows (F), (H), (H+V), (V), attr H=1 V=2. */
int or_prepare_global_ds(const uint8_t *palpix, const uint8_t *active, int T, float *ds, int32_t *tile_idx,
                         uint8_t *attrs) {
    int di = 0;
    uint8_t t[64];
    static const uint8_t order[4] = {0, 1, 3, 2};
    for (int i = 0; i < T; i++) {
        if (!active[i]) continue;
        memcpy(t, palpix + 64 * (size_t)i, 64);
        for (int o = 0; o < 4; o++) {
            if (o == 1) hflip(t);
            if (o == 2) vflip(t);
            if (o == 3) hflip(t);
            for (int j = 0; j < 64; j++) ds[(size_t)di * 64 + j] = (float)t[j];
            tile_idx[di] = i;
            attrs[di] = order[o];
            di++;
        }
    }
    return di;
}

/* BuildPaletteCorrTriangle main.pas:3855-3867 with CompareEuclideanDCTPtr 659-675. */
double or_palette_corr(const double *centroids, int P, double *corrs) {
    double highest = 0.0;
    for (int j = 0; j < P; j++)
        for (int i = 0; i < P; i++) {
            const double *a = centroids + 192 * (size_t)j, *b = centroids + 192 * (size_t)i;
            double r = 0.0;
            for (int k = 0; k < 192; k++) {
                double t = a[k] - b[k];
                r += t * t;
            }
            corrs[(size_t)j * P + i] = r;
            if (!isnan(r)) highest = (highest > r) ? highest : r; /* Max(HighestCorr, r) */
        }
    return highest;
}

/* PrepareFrameTiling.UseOne main.pas:3802-3853 (+ DoBuild 3869-3881).  used: P x T x 4 bytes. */
void or_mark_used(const float *gds, int gn, const int32_t *g_tile, const uint8_t *g_attr, const int32_t *item_pal,
                  const int32_t *item_tile, int nitems, const uint8_t *palpix, int T, int P, int quality,
                  const double *corrs, double highest, double paltol, int kd_order, uint8_t *used) {
    uint8_t *seen = (uint8_t *)calloc((size_t)P * T, 1);
    /* the distinct (pal, tile) items in first-seen order, their 64-index query lines and k = 8 results */
    int *ip = (int *)malloc(sizeof(int) * (size_t)(nitems > 0 ? nitems : 1));
    int *itl = (int *)malloc(sizeof(int) * (size_t)(nitems > 0 ? nitems : 1));
    int nd = 0;
    for (int it = 0; it < nitems; it++) {
        int p = item_pal[it], ti = item_tile[it];
        if (seen[(size_t)p * T + ti]) continue;
        seen[(size_t)p * T + ti] = 1;
        ip[nd] = p;
        itl[nd] = ti;
        nd++;
    }
    float *lines = (float *)malloc(sizeof(float) * 64 * (size_t)(nd > 0 ? nd : 1));
    int *ridx = (int *)malloc(sizeof(int) * 8 * (size_t)(nd > 0 ? nd : 1));
    float *rerr = (float *)malloc(sizeof(float) * 8 * (size_t)(nd > 0 ? nd : 1));
    for (int j = 0; j < nd; j++)
        for (int i = 0; i < 64; i++) lines[(size_t)j * 64 + i] = (float)palpix[(size_t)itl[j] * 64 + i];
    if (kd_order && gn > 0) {  /* ann_kdtree_search_multi on FGlobalDS.KDT (main.pas:3779,3830) */
        void *kd = or_kdtree_build(gds, gn, 64);
        or_kdtree_search_multi_batch(kd, lines, nd, 8, ridx, rerr, 8);
        or_kdtree_free(kd);
    } else {
        for (int j = 0; j < nd; j++) or_knn(gds, gn, 64, lines + (size_t)j * 64, 8, ridx + 8 * j, rerr + 8 * j);
    }
    for (int j = 0; j < nd; j++) {
        const int p = ip[j];
        const int *idxs = ridx + 8 * (size_t)j;
        const float *errs = rerr + 8 * (size_t)j;
        float last = INFINITY;
        for (int i = 0; i < 8; i++) {
            if (errs[i] == last) continue;
            last = errs[i];
            int idx = idxs[i];
            if (idx < 0) continue; /* k > n: ANN would have aborted */
            size_t cell = (size_t)g_tile[idx] * 4 + g_attr[idx];
            if (quality == 0) {
                used[(size_t)p * T * 4 + cell] = 1;
            } else if (quality == 1) {
                for (int pp = 0; pp < P; pp++)
                    if (corrs[(size_t)pp * P + p] < paltol * highest) used[(size_t)pp * T * 4 + cell] = 1;
            } else {
                for (int pp = 0; pp < P; pp++) used[(size_t)pp * T * 4 + cell] = 1;
            }
        }
    }
    free(seen);
    free(ip);
    free(itl);
    free(lines);
    free(ridx);
    free(rerr);
}

int or_count_used(const uint8_t *used, int P, int T) {
    int c = 0;
    for (size_t i = 0; i < (size_t)P * T * 4; i++) c += used[i] != 0;
    return c;
}

/* PrepareFrameTiling.DoPsyV main.pas:3883-3919: pal asc, tile asc, vmir F/T, hmir F/T. */
int or_build_ft_dataset(const uint8_t *used, int P, int T, const uint8_t *palpix, const uint8_t *thm,
                        const uint8_t *tvm, const int32_t *palettes, int use_wavelets, int gamma, float *ds,
                        int32_t *tidx, int32_t *pidx, uint8_t *attrs) {
    int di = 0;
    double desc[192];
    for (int p = 0; p < P; p++)
        for (int i = 0; i < T; i++)
            for (int vm = 0; vm < 2; vm++)
                for (int hm = 0; hm < 2; hm++) {
                    if (!used[((size_t)p * T + i) * 4 + (vm << 1 | hm)]) continue;
                    int f = OR_FROM_PAL | (use_wavelets ? OR_WAVELETS : 0);
                    if (hm ^ (thm ? thm[i] : 0)) f |= OR_HMIRROR;
                    if (vm ^ (tvm ? tvm[i] : 0)) f |= OR_VMIRROR;
                    or_psyv(NULL, palpix + 64 * (size_t)i, palettes + 16 * (size_t)p, f, gamma, desc);
                    for (int j = 0; j < 192; j++) ds[(size_t)di * 192 + j] = (float)desc[j];
                    tidx[di] = i;
                    pidx[di] = p;
                    attrs[di] = (uint8_t)(hm | (vm << 1));
                    di++;
                }
    return di;
}

/* DoFrameTiling main.pas:3992-4047 (query descriptor 4023-4025, search 4027, tilemap 4029-4034). */
void or_frame_tiling(const int32_t *frame_rgb, int Q, const float *ds, int M, const int32_t *tidx,
                     const int32_t *pidx, const uint8_t *attrs, int use_wavelets, int gamma, int threads, int kd_order,
                     int32_t *out_tile, int32_t *out_pal, uint8_t *out_h, uint8_t *out_v, float *out_err) {
    float *qs = (float *)malloc(sizeof(float) * 192 * (size_t)Q);
    int *bi = (int *)malloc(sizeof(int) * (size_t)Q);
    double desc[192];
    for (int i = 0; i < Q; i++) {
        or_psyv(frame_rgb + 64 * (size_t)i, NULL, NULL, use_wavelets ? OR_WAVELETS : 0, gamma, desc);
        for (int j = 0; j < 192; j++) qs[(size_t)i * 192 + j] = (float)desc[j];
    }
    if (kd_order && M > 0) {  /* ann_kdtree_search on the keyframe's KDT (main.pas:3961, 4027) */
        void *kd = or_kdtree_build(ds, M, 192);
        or_kdtree_search_batch(kd, qs, Q, bi, out_err, threads);
        or_kdtree_free(kd);
    } else {
        or_nn_batch(ds, M, 192, qs, Q, bi, out_err, threads);
    }
    for (int i = 0; i < Q; i++) {
        int b = bi[i];
        out_tile[i] = b >= 0 ? tidx[b] : -1;
        out_pal[i] = b >= 0 ? pidx[b] : -1;
        out_h[i] = b >= 0 ? (attrs[b] & 1) != 0 : 0;
        out_v[i] = b >= 0 ? (attrs[b] & 2) != 0 : 0;
    }
    free(qs);
    free(bi);
}

/* ------------------------------------------------------------------------------------------
 * Smooth: btnSmoothClick main.pas:1338-1370, DoTemporalSmoothing 4071-4119.  Arrays are [F][Q]
 * for ONE keyframe (the KF check at 4081-4082 makes chains keyframe-local).  In/out.
 * ---------------------------------------------------------------------------------------- */
void or_smooth(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
               uint8_t *smoothed, const uint8_t *palpix, const int32_t *palettes, double strength) {
    const double sqrt_factor = 1.0 / (64.0 * 3.0); /* cSqrtFactor 4073 */
    double a[192], b[192];
    for (int i = 1; i < F; i++)
        for (int s = 0; s < Q; s++) {
            size_t c = (size_t)i * Q + s, p = (size_t)(i - 1) * Q + s;
            or_psyv(NULL, palpix + 64 * (size_t)tile[p], palettes + 16 * (size_t)pal[p],
                    OR_FROM_PAL | OR_QWEIGHT | (hm[p] ? OR_HMIRROR : 0) | (vm[p] ? OR_VMIRROR : 0), -1, b);
            or_psyv(NULL, palpix + 64 * (size_t)tile[c], palettes + 16 * (size_t)pal[c],
                    OR_FROM_PAL | OR_QWEIGHT | (hm[c] ? OR_HMIRROR : 0) | (vm[c] ? OR_VMIRROR : 0), -1, a);
            double cmp = 0.0;
            for (int k = 0; k < 192; k++) {
                double t = a[k] - b[k];
                cmp += t * t;
            }
            cmp = sqrt(cmp * sqrt_factor);
            if (fabs(cmp) <= strength) {
                if (tile[c] >= tile[p]) {
                    tile[c] = tile[p];
                    if (tmpidx) tmpidx[c] = tmpidx[p];
                    pal[c] = pal[p];
                    hm[c] = hm[p];
                    vm[c] = vm[p];
                    smoothed[c] = smoothed[p];
                } else {
                    tile[p] = tile[c];
                    if (tmpidx) tmpidx[p] = tmpidx[c];
                    pal[p] = pal[c];
                    hm[p] = hm[c];
                    vm[p] = vm[c];
                    smoothed[p] = smoothed[c];
                }
                smoothed[c] = 1;
            } else {
                smoothed[c] = 0;
            }
        }
}

/* ------------------------------------------------------------------------------------------
 * K-Modes (kmodes.pas).  Dissimilarity as the x86-64 asm computes it (kmodes.pas:341-412):
 *   dis = 2048 * #mismatch(80 B) + W0 + W4, W0/W4 16-bit lanes of pabsb(bytes 0..15) + psadbw.
 * ---------------------------------------------------------------------------------------- */
static inline unsigned abs8(uint8_t r, uint8_t x) {
    int8_t d = (int8_t)(uint8_t)(r - x); /* psubb + pabsb */
    return d < 0 ? (unsigned)(-(int)d) : (unsigned)d;
}

uint64_t or_km_dissim(const uint8_t *r, const uint8_t *x) {
    unsigned mism = 0;
    for (int k = 0; k < 80; k++) mism += r[k] != x[k];
    unsigned slo = 0, shi = 0;
    for (int blk = 16; blk < 80; blk += 16) {
        for (int k = 0; k < 8; k++) slo += (unsigned)abs((int)r[blk + k] - (int)x[blk + k]);
        for (int k = 8; k < 16; k++) shi += (unsigned)abs((int)r[blk + k] - (int)x[blk + k]);
    }
    unsigned w0 = (abs8(r[0], x[0]) + 256u * abs8(r[1], x[1]) + slo) & 0xffffu;
    unsigned w4 = (abs8(r[8], x[8]) + 256u * abs8(r[9], x[9]) + shi) & 0xffffu;
    return ((uint64_t)mism << 11) + w0 + w4;
}

/* The same value with SSE2 on 16-byte blocks (the shape of the reference asm, kmodes.pas:341-412): pcmpeqb +
 * movemask for the mismatch count, psadbw for S_lo / S_hi (its two 8-byte halves).  Used by the argmin and
 * min-distance loops; tests/test_oracle_kats.py checks it against or_km_dissim and the reference asm. */
#if defined(__SSE2__)
#include <emmintrin.h>
static inline uint64_t km_dissim_fast(const uint8_t *r, const uint8_t *x) {
    unsigned eqm = 0;
    __m128i sad = _mm_setzero_si128();
    for (int blk = 0; blk < 80; blk += 16) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(r + blk)), b = _mm_loadu_si128((const __m128i *)(x + blk));
        eqm += (unsigned)__builtin_popcount((unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(a, b)));
        if (blk) sad = _mm_add_epi64(sad, _mm_sad_epu8(a, b));
    }
    const unsigned slo = (unsigned)_mm_cvtsi128_si32(sad), shi = (unsigned)_mm_cvtsi128_si32(_mm_srli_si128(sad, 8));
    const unsigned w0 = (abs8(r[0], x[0]) + 256u * abs8(r[1], x[1]) + slo) & 0xffffu;
    const unsigned w4 = (abs8(r[8], x[8]) + 256u * abs8(r[9], x[9]) + shi) & 0xffffu;
    return ((uint64_t)(80u - eqm) << 11) + w0 + w4;
}
#else
#define km_dissim_fast or_km_dissim
#endif

uint64_t or_km_dissim_fast(const uint8_t *r, const uint8_t *x) { return km_dissim_fast(r, x); }

/* MatchingDissim generic path kmodes.pas:239-250 (not the one that runs on x86-64). */
uint64_t or_km_dissim_generic(const uint8_t *a, const uint8_t *b, int n) {
    uint64_t r = 0;
    for (int i = 0; i < n; i++) {
        if (a[i] != b[i]) r += (uint64_t)1 << 11;
        r += (uint64_t)abs((int)a[i] - (int)b[i]);
    }
    return r;
}

/* GetMinMatchingDissim_Asm kmodes.pas:316-453: argmin with <= (ties -> last), -1 if empty. */
int or_km_get_min(const uint8_t *rows, int count, const uint8_t *item, uint64_t *best) {
    uint64_t b = UINT64_MAX;
    int bi = -1;
    for (int i = 0; i < count; i++) {
        uint64_t d = km_dissim_fast(rows + (size_t)i * 80, item);
        if (d <= b) {
            b = d;
            bi = i;
        }
    }
    if (best) *best = b;
    return bi;
}

/* UpdateMinDistance_Asm kmodes.pas:455-596: strict-less min; the 'used' test is a no-op (567). */
void or_km_update_min_distance(const uint8_t *item, const uint8_t *rows, int count, uint64_t *mindist) {
    for (int i = 0; i < count; i++) {
        uint64_t d = km_dissim_fast(rows + (size_t)i * 80, item);
        if (d < mindist[i]) mindist[i] = d;
    }
}

/* RandInt kmodes.pas:82-86 (Delphi LCG). */
uint32_t or_randint(uint32_t range, uint32_t *seed) {
    *seed = (uint32_t)(*seed * 0x08088405u) + 1u;
    return (uint32_t)(((uint64_t)*seed * (uint64_t)range) >> 32);
}

/* ---- a small pthread parallel-for: the reference runs the K-Modes distance loops on 4 threads per bin
 * (TKModes.Create(4), main.pas:4217; DoGMMD / DoUMD via ProcThreadPool, kmodes.pas:877, 693).  Results do
 * not depend on the split: every item is computed independently. ---- */
typedef void (*pf_fn)(void *ctx, int begin, int end);
typedef struct {
    pf_fn fn;
    void *ctx;
    int begin, end;
} pf_job;

static void *pf_run(void *p) {
    pf_job *j = (pf_job *)p;
    j->fn(j->ctx, j->begin, j->end);
    return NULL;
}

static int g_km_threads = 1;
void or_set_threads(int t) { g_km_threads = t < 1 ? 1 : (t > 64 ? 64 : t); }

static void parallel_for(int count, long work_per_item, pf_fn fn, void *ctx) {
    int t = g_km_threads;
    if ((long)count * work_per_item < (1L << 22)) t = 1; /* not worth a thread start */
    if (t > count) t = count;
    if (t <= 1) {
        if (count > 0) fn(ctx, 0, count);
        return;
    }
    pthread_t th[64];
    pf_job jobs[64];
    for (int i = 0; i < t; i++) {
        jobs[i] = (pf_job){fn, ctx, (int)((long)count * i / t), (int)((long)count * (i + 1) / t)};
        if (i) pthread_create(&th[i], NULL, pf_run, &jobs[i]);
    }
    pf_run(&jobs[0]);
    for (int i = 1; i < t; i++) pthread_join(th[i], NULL);
}

typedef struct {
    const uint8_t *item, *rows;
    uint64_t *mindist;
} umd_ctx;
static void umd_part(void *c, int b, int e) {
    umd_ctx *u = (umd_ctx *)c;
    or_km_update_min_distance(u->item, u->rows + (size_t)b * 80, e - b, u->mindist + b);
}

typedef struct {
    const uint8_t *cent, *X;
    int K, A;
    int32_t *clust;
    uint64_t *dis;
} gmmd_ctx;
static void gmmd_part(void *c, int b, int e) {
    gmmd_ctx *g = (gmmd_ctx *)c;
    for (int i = b; i < e; i++) g->clust[i] = or_km_get_min(g->cent, g->K, g->X + (size_t)i * g->A, &g->dis[i]);
}

typedef struct {
    const uint8_t *X;
    int N, A, K, M;
    int32_t *memb;
    uint8_t *cent;
    int32_t *freq; /* K x A x M */
    int32_t *csize;
} km_state;

/* GetMaxValueIndex kmodes.pas:149-161: first max. */
static int max_value_index(const int32_t *arr, int n) {
    int r = -1;
    int32_t best = INT32_MIN;
    for (int i = 0; i < n; i++)
        if (arr[i] > best) {
            best = arr[i];
            r = i;
        }
    return r;
}

/* MovePointCat kmodes.pas:778-806 */
static void move_point_cat(km_state *s, int ipoint, int to, int from) {
    const uint8_t *pt = s->X + (size_t)ipoint * s->A;
    s->memb[ipoint] = to;
    s->csize[to]++;
    s->csize[from]--;
    for (int a = 0; a < s->A; a++) {
        int cur = pt[a];
        int32_t *tc = s->freq + ((size_t)to * s->A + a) * s->M;
        int32_t *fc = s->freq + ((size_t)from * s->A + a) * s->M;
        tc[cur]++;
        int ccv = s->cent[(size_t)to * s->A + a];
        if (tc[ccv] < tc[cur]) s->cent[(size_t)to * s->A + a] = (uint8_t)cur;
        fc[cur]--;
        if (s->cent[(size_t)from * s->A + a] == cur) s->cent[(size_t)from * s->A + a] = (uint8_t)max_value_index(fc, s->M);
    }
}

/* InitFarthestFirst kmodes.pas:698-776 */
static void init_farthest_first(km_state *s, int init_point) {
    uint64_t *mind = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)s->N);
    uint8_t *used = (uint8_t *)calloc((size_t)s->N, 1);
    memset(s->cent, 0xff, (size_t)s->K * s->A);
    for (int i = 0; i < s->N; i++) mind[i] = UINT64_MAX;
    int f = init_point;
    memcpy(s->cent, s->X + (size_t)f * s->A, (size_t)s->A);
    used[f] = 1;
    umd_ctx u = {s->X + (size_t)f * s->A, s->X, mind};
    parallel_for(s->N, 80, umd_part, &u);
    for (int c = 1; c < s->K; c++) {
        uint64_t mx = 0;
        f = -1;
        for (int i = 0; i < s->N; i++)
            if (mind[i] >= mx && !used[i]) {
                mx = mind[i];
                f = i;
            }
        if (f < 0) break; /* K > N: the reference would fault here */
        memcpy(s->cent + (size_t)c * s->A, s->X + (size_t)f * s->A, (size_t)s->A);
        used[f] = 1;
        u.item = s->X + (size_t)f * s->A;
        parallel_for(s->N, 80, umd_part, &u);
    }
    free(mind);
    free(used);
}

/* KModesIter kmodes.pas:845-915 (960-point bins against the current centroid snapshot). */
static int kmodes_iter(km_state *s, uint32_t *seed, uint64_t *cost) {
    const int BIN = 960;
    int moves = 0;
    uint64_t acc = 0;
    int32_t *clust = (int32_t *)malloc(sizeof(int32_t) * (size_t)s->N);
    uint64_t *dis = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)s->N);
    int32_t *choices = (int32_t *)malloc(sizeof(int32_t) * (size_t)s->N);
    for (int b0 = 0; b0 < s->N; b0 += BIN) {
        int last = (b0 + BIN < s->N ? b0 + BIN : s->N) - 1;
        gmmd_ctx g = {s->cent, s->X + (size_t)b0 * s->A, s->K, s->A, clust + b0, dis + b0};
        parallel_for(last - b0 + 1, 80L * s->K, gmmd_part, &g);
        for (int i = b0; i <= last; i++) {
            acc += dis[i];
            if (s->memb[i] != clust[i]) {
                moves++;
                int old = s->memb[i];
                move_point_cat(s, i, clust[i], old);
                if (s->csize[old] == 0) { /* CountClusterMembers(old_clust) = 0 */
                    int from = 0, mc = 0;  /* GetMaxClusterMembers 631-669: '>=' -> last */
                    for (int c = 0; c < s->K; c++)
                        if (s->csize[c] >= mc) {
                            mc = s->csize[c];
                            from = c;
                        }
                    int cnt = 0;
                    for (int j = 0; j < s->N; j++)
                        if (s->memb[j] == from) choices[cnt++] = j;
                    int r = choices[or_randint((uint32_t)cnt, seed)];
                    move_point_cat(s, r, old, from);
                }
            }
        }
    }
    free(clust);
    free(dis);
    free(choices);
    *cost = acc;
    return moves;
}

/* ComputeKModes kmodes.pas:917-1060, ANumInit <= 0 path (start = -ANumInit, l.949-953). */
int or_kmodes(const uint8_t *X, int N, int A, int K, int start, int modalities, int32_t *labels,
              uint8_t *centroids, int *n_iter, uint64_t *cost_out) {
    uint32_t seed = 0x42381337u;
    km_state s = {X, N, A, K, modalities, labels, centroids, NULL, NULL};
    s.freq = (int32_t *)calloc((size_t)K * A * modalities, sizeof(int32_t));
    s.csize = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    init_farthest_first(&s, start);
    {  /* DoGMMD over all points (kmodes.pas:984-997) */
        uint64_t *d0 = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(N > 0 ? N : 1));
        gmmd_ctx g = {centroids, X, K, A, labels, d0};
        parallel_for(N, 80L * K, gmmd_part, &g);
        free(d0);
    }
    for (int i = 0; i < N; i++) s.csize[labels[i]]++;
    for (int i = 0; i < N; i++)
        for (int a = 0; a < A; a++) s.freq[((size_t)labels[i] * A + a) * modalities + X[(size_t)i * A + a]]++;
    for (int k = 0; k < K; k++) {
        if (s.csize[k] == 0) {
            for (int a = 0; a < A; a++) centroids[(size_t)k * A + a] = X[(size_t)or_randint((uint32_t)N, &seed) * A + a];
        } else {
            for (int a = 0; a < A; a++)
                centroids[(size_t)k * A + a] = (uint8_t)max_value_index(s.freq + ((size_t)k * A + a) * modalities, modalities);
        }
    }
    int itr = 0, conv = 0;
    uint64_t cost = UINT64_MAX, ncost = 0;
    while (!conv) {
        itr++;
        int moves = kmodes_iter(&s, &seed, &ncost);
        conv = (ncost >= cost) || (moves == 0);
        cost = ncost;
    }
    if (n_iter) *n_iter = itr;
    if (cost_out) *cost_out = cost;
    free(s.freq);
    free(s.csize);
    return K;
}

/* ------------------------------------------------------------------------------------------
 * GlobalTiling driver (main.pas:4142-4370) + MakeTilesUnique (2555-2612) + ReindexTiles (4483-4527).
 * ---------------------------------------------------------------------------------------- */
/* EqualQualityTileCount main.pas:722-725: FPC Round = banker's rounding; log2 from FPC's Math unit,
 * ln(x) * 1.4426950408889634079 (1/ln 2), not ln(x) / ln(2).  (FPC's own ln may still differ from glibc's
 * log by an ulp; tests/test_global_tiling.py shows no tile count up to 2^22 is that close to a .5.) */
int or_eqtc(double n) { return (int)nearbyint(sqrt(n) * (log(1.0 + n) * 1.4426950408889634079)); }

/* WriteTileDatasetLine main.pas:4167-4183 + GetTilePalZoneThres 4142-4165 (ZoneCount 16). */
int or_tile_dataset_line(const uint8_t *pp, int palsize, uint8_t *line) {
    uint8_t acc[64];
    memset(acc, 0, sizeof(acc));
    const int zc = 16;
    for (int i = 0; i < 64; i++) {
        line[i] = pp[i];
        acc[pp[i] * zc / palsize]++;
    }
    int res = 64;
    for (int i = 0; i < zc; i++) {
        int v = 64 - acc[i];
        res = res < v ? res : v;
        line[64 + i] = acc[i] > (palsize / zc);
    }
    return res;
}

/* MergeTiles main.pas:3688-3712 */
static void merge_tiles(const int32_t *idx, int cnt, int best, uint8_t *palpix, uint8_t *active, int32_t *use_count,
                        int32_t *merge_index) {
    for (int k = 0; k < cnt; k++) {
        int j = idx[k];
        if (j == best) continue;
        use_count[best] += use_count[j];
        active[j] = 0;
        merge_index[j] = best;
        memset(palpix + 64 * (size_t)j, 0, 64);
    }
}

static int cmp_dword_tiles_ctx_T;
static const uint8_t *cmp_pp;
/* CompareTilePalPixels main.pas:2546-2553: CompareDWord over 16 little-endian dwords; stable
 * tie order by original index (canonical; TFPList.Sort is unstable: SURVEY.md 8(f)-1). */
static int cmp_tiles(const void *pa, const void *pb) {
    int a = *(const int *)pa, b = *(const int *)pb;
    const uint8_t *ta = cmp_pp + 64 * (size_t)a, *tb = cmp_pp + 64 * (size_t)b;
    for (int i = 0; i < 16; i++) {
        uint32_t da, db;
        memcpy(&da, ta + 4 * i, 4);
        memcpy(&db, tb + 4 * i, 4);
        if (da != db) return da < db ? -1 : 1;
    }
    return a < b ? -1 : (a > b);
}

void or_make_tiles_unique(int T, uint8_t *palpix, uint8_t *active, int32_t *use_count, int32_t *merge_index) {
    (void)cmp_dword_tiles_ctx_T;
    int *lst = (int *)malloc(sizeof(int) * (size_t)(T > 0 ? T : 1));
    int n = 0;
    for (int i = 0; i < T; i++) {
        merge_index[i] = -1;
        if (active[i]) lst[n++] = i;
    }
    cmp_pp = palpix;
    qsort(lst, (size_t)n, sizeof(int), cmp_tiles);
    /* DoOneMerge (main.pas:2562-2572) closes the group [firstSameIdx, i) at each key change; the final call
     * runs with i := sortList.Count - 1 (main.pas:2604-2605), so the LAST group never includes its last
     * sorted member (a 2-member last group does not merge at all): reproduced, not fixed. */
    int first = 0;
    for (int i = 1; i < n; i++) {
        if (memcmp(palpix + 64 * (size_t)lst[i - 1], palpix + 64 * (size_t)lst[i], 64) != 0) {
            if (i - first >= 2) merge_tiles(lst + first, i - first, lst[first], palpix, active, use_count, merge_index);
            first = i;
        }
    }
    if (n > 0 && (n - 1) - first >= 2)
        merge_tiles(lst + first, (n - 1) - first, lst[first], palpix, active, use_count, merge_index);
    free(lst);
}

/* ReindexTiles main.pas:4483-4527: new order = (UseCount desc, old index asc).  idx_map[old] = new. */
static const int32_t *cmp_uc;
static int cmp_reindex(const void *pa, const void *pb) {
    int a = *(const int *)pa, b = *(const int *)pb;
    if (cmp_uc[a] != cmp_uc[b]) return cmp_uc[a] > cmp_uc[b] ? -1 : 1;
    return a < b ? -1 : (a > b);
}
int or_reindex(int T, const uint8_t *active, const int32_t *use_count, int32_t *idx_map) {
    int *lst = (int *)malloc(sizeof(int) * (size_t)(T > 0 ? T : 1));
    int n = 0;
    for (int i = 0; i < T; i++) {
        idx_map[i] = -1;
        if (active[i]) lst[n++] = i;
    }
    cmp_uc = use_count;
    qsort(lst, (size_t)n, sizeof(int), cmp_reindex);
    for (int i = 0; i < n; i++) idx_map[lst[i]] = i;
    free(lst);
    return n;
}

/* DoGlobalTiling main.pas:4256-4331 + DoKModes 4195-4254 (KModes per palette bin, medoid merge).
 * Tiles are updated in place; the caller applies merge_index to tilemaps (FinishMergeTiles). */
int or_global_tiling(int T, uint8_t *palpix, uint8_t *active, int32_t *use_count, int32_t *merge_index,
                     const int32_t *dith_pal, int P, int palsize, int desired, int restart, int32_t *k_per_bin) {
    int *cnt = (int *)calloc((size_t)P, sizeof(int));
    int *start = (int *)malloc(sizeof(int) * (size_t)P);
    int *best = (int *)malloc(sizeof(int) * (size_t)P);
    for (int p = 0; p < P; p++) {
        start[p] = -restart;
        best[p] = 0x7fffffff;
    }
    for (int i = 0; i < T; i++)
        if (active[i]) cnt[dith_pal[i]]++;
    uint8_t **ds = (uint8_t **)calloc((size_t)P, sizeof(uint8_t *));
    int **tix = (int **)calloc((size_t)P, sizeof(int *));
    for (int p = 0; p < P; p++) {
        ds[p] = (uint8_t *)malloc((size_t)(cnt[p] + 1) * 80);
        tix[p] = (int *)malloc(sizeof(int) * (size_t)(cnt[p] + 1));
        cnt[p] = 0;
    }
    for (int i = 0; i < T; i++) {
        if (!active[i]) continue;
        int s = dith_pal[i];
        uint8_t *line = ds[s] + (size_t)cnt[s] * 80;
        or_tile_dataset_line(palpix + 64 * (size_t)i, palsize, line);
        tix[s][cnt[s]] = i;
        int acc = 0;
        for (int j = 0; j < 80; j++) acc += line[j];
        if (acc <= best[s]) {
            start[s] = cnt[s];
            best[s] = acc;
        }
        cnt[s]++;
    }
    long dis_cnt = 0;
    for (int p = 0; p < P; p++) dis_cnt += or_eqtc(cnt[p]);
    double share = (double)desired / (double)dis_cnt;
    for (int i = 0; i < T; i++) merge_index[i] = -1; /* InitMergeTiles */
    for (int p = 0; p < P; p++) {
        double kc = ceil(or_eqtc(cnt[p]) * share);
        int K = (int)nearbyint(kc);
        if (k_per_bin) k_per_bin[p] = K;
        if (cnt[p] <= kc) continue;
        int32_t *labels = (int32_t *)malloc(sizeof(int32_t) * (size_t)cnt[p]);
        uint8_t *cent = (uint8_t *)malloc((size_t)K * 80);
        or_kmodes(ds[p], cnt[p], 80, K, start[p], palsize, labels, cent, NULL, NULL);
        uint8_t *tm = (uint8_t *)malloc((size_t)cnt[p] * 80);
        int32_t *tmi = (int32_t *)malloc(sizeof(int32_t) * (size_t)cnt[p]);
        for (int j = 0; j < K; j++) {
            int di = 0;
            for (int i = 0; i < cnt[p]; i++)
                if (labels[i] == j) {
                    memcpy(tm + (size_t)di * 80, ds[p] + (size_t)i * 80, 80);
                    tmi[di++] = tix[p][i];
                }
            if (di >= 2) {
                /* GetMinMatchingDissim(ToMerge, LocCentroids[j]): item = centroid, rows = members */
                int b = or_km_get_min(tm, di, cent + (size_t)j * 80, NULL);
                merge_tiles(tmi, di, tmi[b], palpix, active, use_count, merge_index);
            }
        }
        free(labels);
        free(cent);
        free(tm);
        free(tmi);
    }
    for (int p = 0; p < P; p++) {
        free(ds[p]);
        free(tix[p]);
    }
    free(ds);
    free(tix);
    free(cnt);
    free(start);
    free(best);
    return 0;
}

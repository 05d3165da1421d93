/*
 * tiler_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the b0nefish/tiler tile-search hot path (FrameTiling, Smooth,
 * GlobalTiling K-Modes).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  The product path (libANN.so) never links it.
 *
 * Every function cites the reference file:line it restates.  Numeric rules:
 *   - fp64 descriptor math in source order, no FMA contraction (-ffp-contract=off);
 *   - fp32 ANN distances: t = q-c; dist = dist + t*t, each op rounded (ANN.dll leaf scan);
 *   - K-Modes dissimilarity as the x86-64 asm actually computes it (kmodes.pas:316-453).
 *
 * Parity pins: the K-Modes dissimilarity / argmin / min-distance update are pinned against
 * the reference's own asm assembled from kmodes.pas (oracle/build_ref_asm.sh -> oracle/_ref).
 * The descriptor, FT and Smooth paths have no reference fixture (no FPC, ANN.dll is a PE):
 * they are pinned by known-answer tests (tests/golden) derived from the formulas.  Ties follow
 * ANN 1.1.2's kd-tree search (ann_kdtree.c, the published algorithm restated; kd_order = 1), or
 * the lowest candidate index (kd_order = 0, the opt-in rule).
 */
#ifndef TILER_ORACLE_H
#define TILER_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_TILE_W 8
#define OR_DESC_D 192
#define OR_KM_ATTRS 80

/* flags for or_psyv (ComputeTilePsyVisFeatures arguments, main.pas:2997) */
#define OR_FROM_PAL 1
#define OR_WAVELETS 2
#define OR_LAB 4 /* UseLAB: RGBToLAB instead of RGBToYUV (PrepareDitherTiles, main.pas:2120) */
#define OR_QWEIGHT 8
#define OR_HMIRROR 16
#define OR_VMIRROR 32

void or_init(void);
void or_set_gamma(double g0, double g1);
const double *or_dct_lut(void);
const double *or_gamma_lut(void); /* [3][256], row g+1 for g = -1..1 */

void or_psyv(const int32_t *rgb, const uint8_t *palpix, const int32_t *pal, int flags, int gamma, double *out);
void or_psyv_batch(int n, const int32_t *rgb, const uint8_t *palpix, const int32_t *pals, const int32_t *pal_of,
                   const uint8_t *flags_per, int flags, int gamma, double *out);

float or_dist(const float *a, const float *b, int d);
int or_nn(const float *data, int n, int d, const float *q, float *err);
void or_knn(const float *data, int n, int d, const float *q, int k, int *idx, float *err);
void or_nn_batch(const float *data, int n, int d, const float *q, int nq, int *idx, float *err, int threads);

/* ANN 1.1.2 kd-tree (ANN_KD_STD, bucket 1, eps 0): the reference's CPU search (ann_kdtree.c). */
void *or_kdtree_build(const float *data, int n, int d);
void *or_kdtree_build_bs(const float *data, int n, int d, int bs);
void or_kdtree_free(void *t);
long or_kdtree_search_batch(void *t, const float *q, int nq, int *idx, float *err, int threads);
long or_kdtree_search_multi_batch(void *t, const float *q, int nq, int k, int *idx, float *err, int threads);
void or_kdtree_pri_search_batch(void *t, const float *q, int nq, float eps, int *idx, float *err);
void or_kdtree_positions(void *t, int *pos);
void or_kdtree_splits(void *t, int *cd, float *cv, float *lo, float *hi);

/* LZMA-alone decoder (lzma_dec.c): decoded size, -1 corrupt, -2 out too small; consumed = bytes read. */
long or_lzma_decode(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *consumed);

int or_prepare_global_ds(const uint8_t *palpix, const uint8_t *active, int T, float *ds, int32_t *tile_idx,
                         uint8_t *attrs);
double or_palette_corr(const double *centroids, int P, double *corrs);
/* kd_order: 1 = the k = 8 search through ANN's kd-tree (the reference's tie order), 0 = lowest index */
void or_mark_used(const float *gds, int gn, const int32_t *g_tile, const uint8_t *g_attr, const int32_t *item_pal,
                  const int32_t *item_tile, int nitems, const uint8_t *palpix, int T, int P, int quality,
                  const double *corrs, double highest, double paltol, int kd_order, uint8_t *used);
int or_count_used(const uint8_t *used, int P, int T);
int or_build_ft_dataset(const uint8_t *used, int P, int T, const uint8_t *palpix, const uint8_t *thm,
                        const uint8_t *tvm, const int32_t *palettes, int use_wavelets, int gamma, float *ds,
                        int32_t *tidx, int32_t *pidx, uint8_t *attrs);
void or_frame_tiling(const int32_t *frame_rgb, int Q, const float *ds, int M, const int32_t *tidx,
                     const int32_t *pidx, const uint8_t *attrs, int use_wavelets, int gamma, int threads, int kd_order,
                     int32_t *out_tile, int32_t *out_pal, uint8_t *out_h, uint8_t *out_v, float *out_err);

void or_smooth(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
               uint8_t *smoothed, const uint8_t *palpix, const int32_t *palettes, double strength);

uint64_t or_km_dissim(const uint8_t *row, const uint8_t *item);
uint64_t or_km_dissim_fast(const uint8_t *row, const uint8_t *item); /* SSE2 form of the same value */
uint64_t or_km_dissim_generic(const uint8_t *row, const uint8_t *item, int n);
int or_km_get_min(const uint8_t *rows, int count, const uint8_t *item, uint64_t *best);
void or_km_update_min_distance(const uint8_t *item, const uint8_t *rows, int count, uint64_t *mindist);
uint32_t or_randint(uint32_t range, uint32_t *seed);
void or_set_threads(int threads); /* K-Modes distance loops (the reference: 4 per bin); default 1 */
int or_kmodes(const uint8_t *X, int N, int A, int K, int start, int modalities, int32_t *labels,
              uint8_t *centroids, int *n_iter, uint64_t *cost);

int or_eqtc(double n);
int or_tile_dataset_line(const uint8_t *palpix64, int palsize, uint8_t *line80);
int or_global_tiling(int T, uint8_t *palpix, uint8_t *active, int32_t *use_count, int32_t *merge_index,
                     const int32_t *dith_pal, int P, int palsize, int desired, int restart, int32_t *k_per_bin);
void or_make_tiles_unique(int T, uint8_t *palpix, uint8_t *active, int32_t *use_count, int32_t *merge_index);
int or_reindex(int T, const uint8_t *active, const int32_t *use_count, int32_t *idx_map);

/* Load step keyframe detection (load_kf.c; main.pas:811-828, 1099-1146, 1465-1492) */
double or_interframe_corr(const int32_t *a, const int32_t *b, int tm_w, int tm_h);
void or_interframe_corr_batch(const int32_t *frames, int F, int tm_w, int tm_h, double *corr);
int or_find_keyframes(const double *corr, int F, int tile_map_size, int32_t *kf_of_frame);

/* FinishDitherTiles per-tile work, Thomas Knoll mixing (dither_tk.c; main.pas:1494-1571, 1828-1875, 1998-2055,
 * 4049-4069, QuickSort kmodes.pas:89-136) */
const uint8_t *or_dither_map(void);
void or_tk_plan(const int32_t *pal, int palsize, int32_t col, uint8_t *list);
void or_dither_tiles_tk(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int palsize,
                        uint8_t *palpix, uint8_t *hm, uint8_t *vm);
/* the Yliluoma branch (chkUseTK off; DeviseBestMixingPlanYliluoma main.pas:1573-1826, ASM_DBMP form): the sorted list
 * of one colour (returns its length), and the tiles */
int or_yl_plan(const int32_t *pal, int palsize, int mixed, int32_t col, uint8_t *list);
void or_dither_tiles_yl(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int palsize,
                        int mixed, uint8_t *palpix, uint8_t *hm, uint8_t *vm);


/* palette generation (palette.c): QuantizePalette / DLv3 / FinishQuantizePalette, main.pas:2154-2480 */
int or_dl3quant(const uint8_t *rgb, long npix, int quant_to, int lookup_bpc, int32_t *pal);
void or_rgb_to_hsv(int32_t col, uint8_t *h, uint8_t *s, uint8_t *v);
int32_t or_color_luma(int32_t col);
void or_sort_cmulhs(const int32_t *cols, int n, int32_t *out);
void or_quantize_palettes(const int32_t *rgb, const int32_t *pal_of, const uint8_t *active, long n, int P,
                          int palsize, int bpc, int32_t *pal_out, int32_t *use_count, int32_t *hist, int threads);
void or_finish_quantize_order(const int32_t *use_count, int P, int32_t *lut);

/* detmath.c: fdlibm exp / ln, FPC Math.power (non-integer exponent) */
double or_det_log(double x);
double or_det_exp(double x);
double or_fpc_power(double base, double exponent);

/* kmeans.c: the Dither step's k-means (yakmo call restated; returns the assignment count) */
uint32_t or_mt19937_first(uint32_t seed);
int or_kmeans(const double *X, long n, int d, int k, int max_iter, uint32_t seed, int32_t *labels, double *cent,
              int threads);

#ifdef __cplusplus
}
#endif
#endif

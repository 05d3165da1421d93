/*
 * tiler_ann.h -- C-ABI of libANN.so, the MI355X-native drop-in for the reference's ANN.dll
 * boundary plus batched/device extensions for the FrameTiling, Smooth and GlobalTiling hot path.
 *
 * Reference interface replaced (b0nefish/tiler, /root/reference):
 *   extern.pas:63  function ann_kdtree_create(pa: PPANNFloat; n, dd, bs: Integer; split: TANNsplitRule): PANNkdtree; cdecl;
 *   extern.pas:64  procedure ann_kdtree_destroy(akd: PANNkdtree); cdecl;
 *   extern.pas:65  function ann_kdtree_search(akd: PANNkdtree; q: PANNFloat; eps: TANNFloat; err: PANNFloat): Integer; cdecl;
 *   extern.pas:66  function ann_kdtree_pri_search(akd: PANNkdtree; q: PANNFloat; eps: TANNFloat; err: PANNFloat): Integer; cdecl;
 *   extern.pas:67  function ann_kdtree_search_multi(akd: PANNkdtree; idxs: PInteger; errs: PANNFloat; cnt: Integer;
 *                                                    q: PANNFloat; eps: TANNFloat): Integer; cdecl;
 * Types: TANNFloat = Single (extern.pas:30), Integer = int32, TANNsplitRule = int32 enum (extern.pas:21-28).
 *
 * Semantics kept from ANN 1.1.2: exact nearest neighbours of the fp32
 * squared distance accumulated in dimension order with every operation rounded (no FMA); err =
 * squared distance (no sqrt); k results ascending; among equal distances the candidate ANN's own
 * kd-tree search finds first (split = ANN_KD_STD, bucket size bs: the tree is built exactly as
 * ANN's kd_tree constructor builds it, and the search result is the one annkSearch returns, its
 * box-distance pruning included).  Differences (superset behaviour):
 *   - split = TILER_SPLIT_INDEX_ORDER (100): no tree, equal distances resolve to the lowest index;
 *     the other ANN split rules (1..5, never used by the reference) are rejected;
 *   - eps > 0 is accepted and ignored: the exact answer satisfies every eps bound;
 *   - ann_kdtree_pri_search returns annkPriSearch's answer (the priority search replayed on the GPU: its leaf
 *     visit order by box distance, hence its own choice among equal distances, and its (1 + eps)^2 termination,
 *     so eps > 0 gives ANN's approximate answer there); the reference declares it (extern.pas:66) and never
 *     calls it;
 *   - the dataset rows are copied to device memory at create (ANN borrows pa until destroy);
 *   - no process abort: errors return -1 (or NULL) and tiler_last_error() explains;
 *   - every entry point is thread-safe.  Concurrent single-query calls on one handle (ann_kdtree_search /
 *     _search_multi from many threads: the reference's ProcThreadPool pattern, main.pas:972, 4027, 3830) are
 *     coalesced: callers that arrive while a batch is in flight are searched together as the next batch,
 *     each woken with its own answer (identical to a lone call's); other calls on one handle are serialised.
 * The search runs on the GPU only.  There is no CPU fallback: if the HIP runtime or a gfx950
 * device is missing every call fails with -1 / NULL.
 */
#ifndef TILER_ANN_H
#define TILER_ANN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ann_kdtree ann_kdtree; /* opaque */

/* ---- the reference ANN.dll surface (extern.pas:63-67), symbol- and ABI-identical ---- */
ann_kdtree *ann_kdtree_create(float **pa, int n, int dd, int bs, int split);
void ann_kdtree_destroy(ann_kdtree *akd);
int ann_kdtree_search(ann_kdtree *akd, float *q, float eps, float *err);
int ann_kdtree_pri_search(ann_kdtree *akd, float *q, float eps, float *err);
int ann_kdtree_search_multi(ann_kdtree *akd, int *idxs, float *errs, int cnt, float *q, float eps);

#define TILER_SPLIT_ANN_KD_STD 0     /* ANN_KD_STD (extern.pas:22): the reference's rule */
#define TILER_SPLIT_INDEX_ORDER 100 /* split value: no kd-tree, ties to the lowest index (faster to create) */

/* Create from fp32 rows already in HBM (d_rows[n][dd], copied); e.g. descriptors made by tiler_psyv_batch_dev.
 * ann_kdtree_create_dev = ann_kdtree_create_dev_ex(..., bs = 1, split = ANN_KD_STD, ...) (main.pas:3961). */
ann_kdtree *ann_kdtree_create_dev(const float *d_rows, int n, int dd, void *stream);
ann_kdtree *ann_kdtree_create_dev_ex(const float *d_rows, int n, int dd, int bs, int split, void *stream);

/* ---- batched extensions; host buffers, row-major q[nq][dd] ---- */
/* k = 1 for every query: idx[nq], err[nq].  Returns 0 or -1. */
int ann_kdtree_search_batch(ann_kdtree *akd, const float *q, int nq, float eps, int *idx, float *err);
/* k results per query, ascending by (err, index): idxs[nq][k], errs[nq][k] (missing: -1 / FLT_MAX). k <= 32. */
int ann_kdtree_search_multi_batch(ann_kdtree *akd, const float *q, int nq, int k, float eps, int *idxs, float *errs);
/* nq ann_kdtree_pri_search calls at once (host arrays; idx / err [nq]) */
int ann_kdtree_pri_search_batch(ann_kdtree *akd, const float *q, int nq, float eps, int *idx, float *err);
/* Same with device-resident buffers (HBM) on a HIP stream (NULL = default stream); asynchronous. */
int ann_kdtree_search_batch_dev(ann_kdtree *akd, const float *d_q, int nq, int k, int *d_idx, float *d_err,
                                void *stream);

/* Search statistics of the last call on this handle (shortlist sizes, exact fallbacks). */
typedef struct {
    int64_t queries;
    int64_t fallback_queries;   /* tier 2: shortlist overflowed -> MFMA collect pass + exact rescoring (any number of
                                   queries; the mirror-orbit tier 2 has no per-query candidate limit) */
    int64_t exhaustive_queries; /* tier 3: exhaustive reference-order scan (k > 8, non-finite / fp16-overflowing data,
                                   and > 1024 candidates for a query of the generic, non-orbit tier 2) */
    int32_t exact_integer;    /* 1 when the dataset is small integers: MFMA keys are exact */
    int32_t splits;           /* candidate splits used by the last launch */
    int64_t orbit_groups;     /* mirror orbits found in the dataset (0: mirror-orbit path unavailable) */
    int32_t orbit_search;     /* 1 when the last search ran the mirror-orbit shortlist */
    int32_t orbit_ksteps;     /* 16-deep MFMA k-steps over 32 groups the orbit shortlist issues per query (12 per
                                 block; fewer on blocks of mirror-symmetric tiles, whose zero blocks are skipped) */
    int64_t orbit_expansions; /* TILER_ORBIT_STATS=1 only: 4-entry re-key passes of the orbit rescore */
    int64_t orbit_rescored;   /* TILER_ORBIT_STATS=1 only: candidates rescored with the reference distance */
    int32_t tie_order;        /* 0: ANN kd-tree first-found (ANN_KD_STD), 1: lowest index */
    int32_t kd_levels;        /* levels of the kd-tree build */
    double kd_build_ms;       /* kd-tree build time at create */
    int64_t kd_replayed;      /* queries of the last search replayed exactly (ANN's pruning not vouched for) */
    int64_t flat_queries;     /* queries of the last FrameTiling call in shortlist workgroups made of flat tiles only
                                 (flat tiles are grouped last; such a workgroup runs isotypic block 0 only: 3 k-steps
                                 per candidate block instead of orbit_ksteps / blocks).  Flat tiles that share a
                                 workgroup with non-flat ones are not counted.  0 for searches without flat grouping. */
} tiler_search_stats;
int ann_kdtree_get_stats(ann_kdtree *akd, tiler_search_stats *out);
/* Search batches of at most max_k1 queries (k = 1; default 64) or max_k8 (k <= 8; default 16) -- the coalesced
 * per-tile calls -- run an exhaustive exact scan spread over the whole GPU instead of the MFMA shortlist and its
 * tiers (same answers; 0 disables it, e.g. to test those tiers on small batches).  Process-wide.  0 / -1. */
int tiler_set_scan_limits(int max_k1, int max_k8);
/* Test hook (process-wide): on != 0 makes ANN's pruning check vouch for no result, so every query of every kd-order
 * search takes the exact replay of annkSearch (kd_replay_kernel); answers are identical either way.  0. */
int tiler_debug_force_replay(int on);
/* Test / bench hook (process-wide): on = 0 switches off the k = 1 generic shortlist's exact insertion gate (the query's
 * best key so far bounds what its lists may need), for A/B timing; answers are identical either
 * way.  Default 1.  0. */
int tiler_debug_shortlist_gate(int on);
/* Coalescing counters of the single-query entry points on this handle: calls, batches searched, largest batch. */
int tiler_combine_stats(ann_kdtree *akd, int64_t *calls, int64_t *batches, int32_t *max_batch);
/* Test / bench hook: the reference's per-call pattern timed natively (no interpreter between the calls): the first
 * min(nq, 64) queries as lone calls on one thread (median latency -> *lone_us), then all nq from `threads` native
 * threads calling ann_kdtree_search (k = 1) or ann_kdtree_search_multi (k > 1) once per query on this one handle
 * (query i on thread i % threads) -> *wall_s.  q[nq][dd] host rows; idx / err [nq][k] receive every answer.  0 / -1. */
int tiler_debug_percall_bench(ann_kdtree *akd, const float *q, int nq, int k, int threads, int32_t *idx, float *err,
                              double *wall_s, double *lone_us);
/* Leaf position of every dataset point in ANN's kd-tree (the order of its depth-first scan with every near
 * child LO): pos[n].  -1 when the handle was created with TILER_SPLIT_INDEX_ORDER. */
int tiler_kdtree_positions(ann_kdtree *akd, int32_t *pos);

/* ---- runtime ---- */
/* Binds the library to one HIP device (one process per GPU: device = LOCAL_RANK), or with TILER_ALL_DEVICES to
 * every visible gfx950 device (one process driving the node: the unmodified FreePascal encoder, whose keyframes run
 * concurrently in one process, main.pas:972 / 3961 / 4005-4011).  Optional; the first call of any other entry point
 * binds device 0.  Re-binding differently once bound fails with -1.
 * With all devices bound: ann_kdtree_create puts each new handle on the least loaded device (live dataset bytes,
 * ties to the lowest device), so concurrent keyframes' handles spread over the GPUs with no call-site change;
 * device-buffer entry points (_dev, ann_kdtree_create_dev*) run on the device their buffers live on, and a handle
 * used there from another device (e.g. the global 64-d dataset in tiler_prepare_frame_tiling_dev) is replicated to
 * it on first use (rows peer-copied over xGMI, the identical index built there); every other call of a handle runs
 * on the handle's device.  Host entry points without a handle run on the caller's current device if bound. */
#define TILER_ALL_DEVICES (-1)
int tiler_init(int device);
int tiler_device_count(void);                              /* devices bound (binds device 0 if none yet) */
int tiler_kdtree_device(ann_kdtree *akd);                  /* the device a handle lives on */
/* Copy a handle's index to device (TILER_ALL_DEVICES: to every bound device) now instead of on first use. 0 / -1. */
int tiler_kdtree_replicate(ann_kdtree *akd, int device);
/* The placement rule alone (host only, no device needed): dev_out[i] = the device ann_kdtree_create would give the
 * i-th of n handles of bytes[i] dataset bytes created in order on ndev empty devices (none destroyed).  0 / -1. */
int tiler_placement_plan(int ndev, const int64_t *bytes, int n, int32_t *dev_out);
/* Test hook (process-wide): on != 0 makes the first device-buffer call of a handle (and tiler_kdtree_replicate) build
 * its copy even on the handle's own device, so the replication path (peer copy, index rebuild, maps copy, routing)
 * runs on a one-GPU box; results are identical either way.  Only with TILER_ALL_DEVICES.  0. */
int tiler_debug_force_replicas(int on);
int tiler_shutdown(void);
const char *tiler_last_error(void); /* thread-local message of the last failure */
int tiler_set_gamma(double g0, double g1); /* gGamma main.pas:586 / 1441-1447; rebuilds gGammaCorLut */
/* Kernel timing with HIP events on the launching stream (bench/profiling): enable, then read the
 * summed milliseconds and launch count of one kernel family ("psyv", "nn_prep", "nn_shortlist",
 * "nn_rescore", "nn_exact", "smooth", "kmodes").  Reading synchronises the recorded events. */
int tiler_timing_enable(int on);
double tiler_timing_get(const char *kernel, int *launches);
int tiler_timing_reset(void);

/* ---- PsyV descriptor (ComputeTilePsyVisFeatures main.pas:2997-3177) ----
 * flags: 1 FromPal, 2 UseWavelets, 4 UseLAB (RGBToLAB main.pas:2711-2747, the Dither step's descriptors),
 * 8 QWeighting, 16 HMirror, 32 VMirror.
 * RGB mode: rgb[n][64] (0x00BBGGRR).  Pal mode: palpix[*][64] indexed by tile_of[i] (or i when NULL),
 * palettes[*][16] indexed by pal_of[i] (or 0), per-item extra flags flags_per[i] (or NULL).
 * gamma: -1 (r/255) or 0/1 (gGammaCorLut).  Outputs: out64[n][192] and/or out32[n][192]. */
int tiler_psyv_batch(int n, const int32_t *rgb, int n_tiles, const uint8_t *palpix, const int32_t *tile_of, int n_palettes,
                     const int32_t *palettes,
                     const int32_t *pal_of, const uint8_t *flags_per, int flags, int gamma, double *out64, float *out32);
/* device-pointer variant (every pointer in HBM); asynchronous on stream */
int tiler_psyv_batch_dev(int n, const int32_t *rgb, const uint8_t *palpix, const int32_t *tile_of,
                         const int32_t *palettes, const int32_t *pal_of, const uint8_t *flags_per, int flags, int gamma,
                         double *out64, float *out32, void *stream);

/* ---- FrameTiling (DoFrameTiling main.pas:3992-4047) ----
 * Attach the keyframe dataset's row -> (tile, palette, attrs) maps (TTilingDataset.TRTo*, main.pas:181-189)
 * to a handle created over the keyframe's candidate descriptors. */
int tiler_ft_set_maps(ann_kdtree *akd, const int32_t *tr_tile, const int32_t *tr_pal, const uint8_t *tr_attr);
/* Read them back (host arrays of the handle's n rows), e.g. the candidate set tiler_prepare_frame_tiling_dev built. */
int tiler_ft_get_maps(ann_kdtree *akd, int32_t *tr_tile, int32_t *tr_pal, uint8_t *tr_attr);
/* For Q frame tiles (RGB): query descriptor (UseWavelets, gamma, no mirror) -> fp32 -> exact NN ->
 * tilemap item {GlobalTileIndex, PalIdx, HMirror = attr&1, VMirror = attr&2} + err. Host buffers. */
int tiler_frame_tiling(ann_kdtree *akd, const int32_t *rgb, int Q, int use_wavelets, int gamma, int32_t *out_tile,
                       int32_t *out_pal, uint8_t *out_hm, uint8_t *out_vm, float *out_err);
/* PrepareFrameTiling (main.pas:3791-3967) for one keyframe, on the device: its tilemap items d_item_tile /
 * d_item_pal [n_items] (TFrame.TileMap GlobalTileIndex / PalIdx of every frame tile; -1 = none) -> the distinct
 * (PalIdx, tile) items -> UseOne's k = 8 preselection in global_ds (the handle over PrepareGlobalFT's 64-d rows, its
 * TRTo maps set with tiler_ft_set_maps; ANN's tie order) -> used[palette][tile][attr] (results of equal err after
 * the first skipped, main.pas:3832-3852; quality 0 Fast: the item's palette, 1 Medium: every palette p' with
 * near[p' * n_palettes + p] != 0 -- the host's corr(p', p) < cFTPaletteTol * HighestCorr, BuildPaletteCorrTriangle
 * main.pas:3855-3867 --, 2 Slow: all) -> DoPsyV's candidates in emission order -> their descriptors -> a new
 * search handle over them with its TRTo maps set, ready for tiler_frame_tiling_dev.  The tileset d_palpix[n_tiles]
 * [64], d_thm / d_tvm[n_tiles] (TTile.HMirror / VMirror) and d_palettes[n_palettes][16] are in HBM; near is a host
 * array (Medium only).  Runs on stream (synchronising it twice: the distinct-item and candidate counts); info
 * (optional) returns those counts.  Calls sharing global_ds are serialised on the host and ordered on the device: a
 * call on another stream waits (hipStreamWaitEvent) until the previous call's work that reads the shared scratch has
 * run, so concurrent prepares on different streams are safe.  NULL on error. */
typedef struct {
    int64_t items;      /* distinct (PalIdx, GlobalTileIndex) items searched */
    int64_t candidates; /* KNNSize: candidate descriptors of the keyframe's dataset */
} tiler_prepare_info;
ann_kdtree *tiler_prepare_frame_tiling_dev(ann_kdtree *global_ds, const int32_t *d_item_tile,
                                           const int32_t *d_item_pal, int64_t n_items, const uint8_t *d_palpix,
                                           const uint8_t *d_thm, const uint8_t *d_tvm, int n_tiles,
                                           const int32_t *d_palettes, int n_palettes, int quality, const uint8_t *near,
                                           int use_wavelets, int gamma, void *stream, tiler_prepare_info *info);
/* Same, every buffer in HBM, asynchronous on stream (the benchmarked path): no host synchronisation inside, every
 * data-dependent count (flat tiles, tier-2 / tier-3 queries) stays on the device. */
int tiler_frame_tiling_dev(ann_kdtree *akd, const int32_t *d_rgb, int Q, int use_wavelets, int gamma,
                           int32_t *d_tile, int32_t *d_pal, uint8_t *d_hm, uint8_t *d_vm, float *d_err, void *stream);

/* ---- Smooth (DoTemporalSmoothing main.pas:4071-4119 over one keyframe) ----
 * Items are [F][Q] arrays (F frames of one keyframe, Q tilemap positions), updated in place exactly
 * as btnSmoothClick does after SmoothedTileMap := TileMap.  palpix[T][64], palettes[P][16]. */
int tiler_smooth_keyframe(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                          uint8_t *smoothed, int T, const uint8_t *palpix, int P, const int32_t *palettes,
                          double strength);
/* Same with every array in HBM (tmpidx may be NULL); asynchronous on stream. */
int tiler_smooth_keyframe_dev(int F, int Q, int32_t *d_tile, int32_t *d_tmpidx, int32_t *d_pal, uint8_t *d_hm,
                              uint8_t *d_vm, uint8_t *d_smoothed, const uint8_t *d_palpix, const int32_t *d_palettes,
                              double strength, void *stream);

/* ---- GlobalTiling K-Modes (TKModes.ComputeKModes kmodes.pas:917-1060) ----
 * X[n][nattr] bytes; k clusters; start_point = -ANumInit (the DoKModes call, main.pas:4218); labels[n]
 * (0-based), centroids[k][nattr].  Returns k or -1.  n_iter / cost optional. */
int tiler_kmodes_compute(const uint8_t *X, int n, int nattr, int k, int start_point, int n_modalities,
                         int32_t *labels, uint8_t *centroids, int *n_iter, uint64_t *cost);
/* DoKModes medoids (main.pas:4231-4253): for every cluster j, the member row minimising the K-Modes
 * dissimilarity to centroid j (ties -> last member, as GetMinMatchingDissim); medoid[j] = -1 and
 * counts[j] = 0 for empty clusters.  X[n][80], labels[n] in 0..k-1, centroids[k][80]. */
int tiler_kmodes_medoids(const uint8_t *X, int n, const int32_t *labels, const uint8_t *centroids, int k,
                         int32_t *medoid, int32_t *counts);
/* All of DoGlobalTiling's palette bins in one call (DoKModes per bin, main.pas:4195-4254, which the
 * reference runs concurrently with ProcThreadPool at main.pas:4339): X[N][80] with bin b = rows
 * [bin_off[b], bin_off[b+1]), k[b] clusters and start[b] (bin-local) per bin; labels[N] bin-local,
 * centroids[sum k][80] bin after bin; n_iter[b] / cost[b] optional.  Each bin's result is exactly
 * tiler_kmodes_compute's on that bin alone.  Returns 0 or -1. */
int tiler_kmodes_batch(const uint8_t *X, const int32_t *bin_off, int nbins, const int32_t *k, const int32_t *start,
                       int n_modalities, int32_t *labels, uint8_t *centroids, int32_t *n_iter, uint64_t *cost);
/* The same with X / labels / centroids in HBM (X 16-byte aligned) on a HIP stream (NULL = default);
 * bin_off / k / start / n_iter / cost are host arrays.  Synchronous. */
int tiler_kmodes_batch_dev(const uint8_t *d_X, const int32_t *bin_off, int nbins, const int32_t *k,
                           const int32_t *start, int n_modalities, int32_t *d_labels, uint8_t *d_centroids,
                           int32_t *n_iter, uint64_t *cost, void *stream);
/* Work counters of the last tiler_kmodes_batch[_dev] call (process-wide): the (point, centroid) dissimilarities its
 * assignment launches evaluated (the initial assignment + every chunk step's), and its dependent chunk steps. */
int tiler_kmodes_last_stats(int64_t *assign_pairs, int64_t *chunk_steps);
/* Test hook (process-wide): on != 0 makes the persistent farthest-first launch give up at its first grid barrier,
 * as a barrier that times out on a contended GPU would, so every batch takes the recovery path (state re-initialised,
 * the rounds re-run one launch each).  Results are identical either way.  0. */
int tiler_debug_kmodes_ff_fallback(int on);
/* Medoids of every bin's clusters (as tiler_kmodes_medoids per bin): medoid[sum k] bin-local rows. */
int tiler_kmodes_medoids_batch(const uint8_t *X, const int32_t *bin_off, int nbins, const int32_t *k,
                               const int32_t *labels, const uint8_t *centroids, int32_t *medoid, int32_t *counts);

/* ---- Load-step keyframe detection (btnLoadClick main.pas:1099-1146) ----------------
 * frames[F][tm_h*tm_w][64] int32 0x00BBGGRR (TFrame.Tiles[].RGBPixels, tile-major, as FrameTiling takes
 * them).  corr[F-1] (host): corr[i-1] = ComputeInterFrameCorrelation(frame i-1, frame i) (main.pas:811-828,
 * PearsonCorrelation main.pas:1465-1492 over LoadFrame's FSPixels), bit-identical to the reference's
 * sequential fp64 evaluation.  0 ok, -1 error.  No reference interface exists for this step (it is inline
 * in btnLoadClick); these exports let the Pascal Load step hand its frames over instead. */
int tiler_interframe_correlation(const int32_t *rgb, int F, int tm_w, int tm_h, double *corr);
/* Same with the frames in HBM (16-byte aligned); corr is a host array; synchronous on stream. */
int tiler_interframe_correlation_dev(const int32_t *d_rgb, int F, int tm_w, int tm_h, double *corr, void *stream);
/* The shot-transition split (main.pas:1099-1132): kf_of_frame[F] = keyframe index of each frame.
 * tile_map_size = FTileMapSize.  Returns the keyframe count, or -1. */
int tiler_find_keyframes(const double *corr, int F, int tile_map_size, int32_t *kf_of_frame);

/* ---- Dither step, per tile (FinishDitherTiles main.pas:2482-2544) -------------------------
 * For n frame tiles rgb[n][64] (0x00BBGGRR) and their keyframe palette pal_of[n] (DitheringPalIndex) out of
 * palettes[n_palettes][palsize] (PaletteRGB, palsize a power of two <= 16): DitherTile with Thomas Knoll mixing
 * (the default, main.pas:1998-2055 / 1828-1875) then PrepareTileMirrors (main.pas:4049-4069) ->
 * palpix[n][64] palette indices in canonical orientation, hm/vm[n] (TTile.HMirror / VMirror).
 * Palette generation (yakmo k-means) and DitheringPalIndex selection are not part of this call.  0 / -1. */
int tiler_dither_tiles(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int n_palettes,
                       int palsize, uint8_t *palpix, uint8_t *hm, uint8_t *vm);
/* Same with every array in HBM; asynchronous on stream. */
int tiler_dither_tiles_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes,
                           int n_palettes, int palsize, uint8_t *d_palpix, uint8_t *d_hm, uint8_t *d_vm, void *stream);
/* The same step with Yliluoma mixing instead (chkUseTK unchecked, main.lfm:272-282): DitherTile's other branch
 * (main.pas:2055-2067) with DeviseBestMixingPlanYliluoma (main.pas:1573-1826, the ASM_DBMP form the reference build
 * compiles), mixed_colors = FY2MixedColors (cbxYilMix: 1, 2, 4 (the form's default), 8, 16; here 1..64), palsize
 * 1..16 (any size).  Then PrepareTileMirrors as above.  0 / -1. */
int tiler_dither_tiles_yliluoma(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes,
                                int n_palettes, int palsize, int mixed_colors, uint8_t *palpix, uint8_t *hm,
                                uint8_t *vm);
int tiler_dither_tiles_yliluoma_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes,
                                    int n_palettes, int palsize, int mixed_colors, uint8_t *d_palpix, uint8_t *d_hm,
                                    uint8_t *d_vm, void *stream);

/* ---- Dither step, palette generation (QuantizePalette / FinishQuantizePalette) ------------
 * QuantizePalette with the default Dennis Lee v3 quantizer (chkUseDL3, main.pas:2154-2254 -> dl3quant,
 * dlquant/quantizer.c:437-663) for n_palettes (keyframe, palette) pairs at once: tiles rgb[n_tiles][64] (0x00BBGGRR,
 * each keyframe's frames in order), pal_of[n_tiles] the pair of each tile (DitheringPalIndex, stacked over
 * keyframes as kf * FPaletteCount + palette; out-of-range indices are skipped), active[n_tiles] or NULL (all
 * Active) -> palettes[n_palettes][palsize] (PaletteIndexes: the palsize DLv3 colours sorted by CompareCMULHS,
 * main.pas:2413-2417; 0 beyond a table that has fewer colours), use_count[n_palettes] (PaletteUseCount.UseCount),
 * colors[n_palettes] or NULL (the DLv3 colour-table size of each pair).  lookup_bpc = cbxDLBPC (7 by default,
 * 1..8).  Outputs are host arrays in both forms.  0 / -1. */
int tiler_quantize_palettes(long n_tiles, const int32_t *rgb, const int32_t *pal_of, const uint8_t *active,
                            int n_palettes, int palsize, int lookup_bpc, int32_t *palettes, int32_t *use_count,
                            int32_t *colors);
int tiler_quantize_palettes_dev(long n_tiles, const int32_t *d_rgb, const int32_t *d_pal_of, const uint8_t *d_active,
                                int n_palettes, int palsize, int lookup_bpc, int32_t *palettes, int32_t *use_count,
                                int32_t *colors, void *stream);
/* Test hook (process-wide) for the DLv3 merges: at most list_cap listed recount_next entries are kept in LDS
 * (list_cap <= 0 or above the built-in 1024 restores 1024); a smaller cap runs the global-memory overflow and the
 * multi-batch path on small tables.  Results are identical for every cap.  0. */
int tiler_debug_dl3(int list_cap);
/* PrepareDitherTiles for one keyframe (main.pas:2097-2152): ComputeTilePsyVisFeatures(UseLAB, use_wavelets,
 * gamma) of its n_tiles RGB tiles (frame order), then the k-means of yakmo_create(n_palettes, 1, MaxInt, k-means++,
 * seed, no normalisation) -> labels[n_tiles] (DitheringPalIndex), centroids[n_palettes][192] (PaletteCentroids),
 * *iterations (Lloyd assignments).  yakmo.dll is binary-only: the k-means is its published algorithm written out
 * exactly (DESIGN.md "Dither: palette generation"), not pinned to the DLL.  max_iter <= 0 means unbounded
 * (MaxInt).  Fewer than 2 tiles or palettes: labels 0, centroids 0.  Host arrays / device pointers.  0 / -1. */
int tiler_prepare_dither_tiles(long n_tiles, const int32_t *rgb, int n_palettes, int gamma, int use_wavelets,
                               int max_iter, uint32_t seed, int32_t *labels, double *centroids, int *iterations);
int tiler_prepare_dither_tiles_dev(long n_tiles, const int32_t *d_rgb, int n_palettes, int gamma, int use_wavelets,
                                   int max_iter, uint32_t seed, int32_t *d_labels, double *d_centroids,
                                   int *iterations, void *stream);
/* The k-means alone over X[n][d] (d <= 192, fp64, host arrays). */
int tiler_kmeans(const double *X, long n, int d, int k, int max_iter, uint32_t seed, int32_t *labels,
                 double *centroids, int *iterations);
/* FinishQuantizePalette's order of one keyframe's palettes (main.pas:2444-2455): the reference QuickSort
 * (kmodes.pas:89-136) by use count, descending -> lut[old palette] = new palette.  0 / -1. */
int tiler_finish_quantize_order(int n_palettes, const int32_t *use_count, int32_t *lut);

/* ---- GTM keyframe stream compression (host code) ---------------------------------------------------
 * Replaces LZCompress (extern.pas:202-240: temp file + external `lzma.exe e src dst -lc8 -eos`, called
 * per keyframe by SaveStream main.pas:4734).  Writes an LZMA-alone stream (13-byte header: properties
 * (pb*5+lp)*9+lc, dictionary size u32, uncompressed size u64 = all ones when eos != 0) into dst.
 * dst == NULL: only *out_len (the exact size) is computed; cap too small: -1 with *out_len = size needed.
 * 0 ok, -1 error (tiler_last_error). */
int tiler_lzma_encode(const uint8_t *src, size_t n, int lc, int lp, int pb, uint32_t dict_size, int eos,
                      uint8_t *dst, size_t cap, size_t *out_len);

#ifdef __cplusplus
}
#endif
#endif

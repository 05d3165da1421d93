// nn_search.hpp -- exact nearest-neighbour search on gfx950 (internal interface).
#pragma once
#include <mutex>
#include <vector>

#include "kdtree.hpp"
#include "tiler_common.hpp"

namespace tiler {

// dataset statistics reduced on device (norm bounds in the scaled space, see nn_search.hip)
struct DsStat {
    unsigned long long max_n2_bits;  // max ||c||^2 (double bits; positive doubles order like u64)
    unsigned long long max_h2_bits;  // max ||fp16(c)||^2
    unsigned long long max_e2_bits;  // max ||c - fp16(c)||^2
    unsigned long long max_abs_bits; // max |c| (double bits)
    unsigned int not_int;            // any value not a small integer (|v| <= 2048)
    unsigned int bad;                // any non-finite value or fp16 overflow
    unsigned int pad[2];
};

// per-query statistics (written by the query prep kernel)
struct QStat {
    double n2;     // ||q||^2 (scaled space)
    double hn;     // ||fp16(q)||
    double en;     // ||q - fp16(q)||
    int flags;     // bit0: integer query, bit1: bad (non-finite / fp16 overflow) -> exact path
    int pad;
};

struct OrbitIndex;  // orbit.hpp

struct SearchScratch {
    void *qfrag = nullptr;
    QStat *qstat = nullptr;
    float *key = nullptr;
    int *idx = nullptr;
    int *fb_list = nullptr;
    int *fb_count = nullptr;  // [2]: count, pad
    float *qrows = nullptr;   // fp32 query rows (frame-tiling path: descriptors)
    void *qfrag16 = nullptr;  // query fragments, 16-row layout
    float *thr = nullptr;     // tier-2 thresholds [nq]
    float2 *gate = nullptr;   // [nq] the generic k = 1 shortlist's insertion gate: T(kk) = (kk + x) * b + y (gate16_kernel)
    int *ex_list = nullptr;   // tier-3 list [nq]
    int *ccnt = nullptr;      // generic tier-2 collect counts [TIER2_MAX] (one chunk)
    int *cbuf = nullptr;      // generic tier-2 collect buffers [TIER2_MAX][TIER2_CAP]
    unsigned long long *t2best = nullptr;  // [nq] orbit tier 2: (distance, ANN rank) minimum per tier-2 slot
    int *kd_list = nullptr;   // [nq] queries the ANN pruning check sends to the exact replay
    int *kd_count = nullptr;  // [1]
    float *kd_rootbox = nullptr;  // [nq] annBoxDistance of each query to the kd-tree's enclosing box
    uint8_t *kd_done = nullptr;   // [nq] 1: the pair pass already checked this query's winner
    // FrameTiling: flat tiles moved last (their descriptors have only isotypic block 0)
    int *fperm = nullptr, *fbcnt = nullptr, *fcnt = nullptr;  // [Q] new -> original, [blocks], [1] non-flat count
    uint8_t *fflag = nullptr;
    int *fidx = nullptr;
    float *ferr = nullptr;
    int32_t *ftile = nullptr, *fpal = nullptr;
    uint8_t *fhm = nullptr, *fvm = nullptr;
    size_t cap_q = 0, cap_keys = 0, cap_rows = 0, cap_flat = 0;
};

struct NNIndex {
    int n = 0, d = 0, S = 0, nblk = 0;
    float scale = 1.0f;         // power of two applied before the fp16 split (keeps |v| <= 16384)
    double maxN = 0, maxH = 0, maxE = 0, max_abs = 0;
    bool exact_int = false;
    int perm = 0;               // 1: candidate rows spread over accumulator lanes (row_perm), float data
    const int *flat_cnt = nullptr; // FrameTiling call in progress: device count of non-flat queries (flat ones last)
    float *d_rows = nullptr;    // [n][d] fp32 (exact rescoring)
    float *d_rowsT = nullptr;   // [ceil(n/64)][d/4][64] float4 row-interleaved copy (k = 1 small-batch scan, built on
                                // first use; null on mirror-orbit indexes, which scan their base rows)
    void *d_frag = nullptr;     // [nblk][S][64][8] fp16, MFMA A-operand fragment order
    float *d_nc = nullptr;      // [nblk][32] ||c||^2 in accumulator-row order (+inf on padding rows)
    float *d_seed = nullptr;    // [nblk][32] -||c||^2/2, same order (-inf on padding rows)
    // 16-row layout for the 16x16x32 shortlist (float datasets of 161..192 dims; S16 = 0 if absent)
    int S16 = 0, nblk16 = 0;
    void *d_frag16 = nullptr;   // [nblk16][S16][64][8] fp16
    float *d_seed16 = nullptr;  // [nblk16][16] -||c||^2/2 by A row
    int32_t *d_tr_tile = nullptr, *d_tr_pal = nullptr;
    uint8_t *d_tr_attr = nullptr;
    SearchScratch scratch;
    std::mutex mu;
    long long last_queries = 0, last_fallback = 0;
    int last_splits = 0;
    // flat_queries of the last search (tiler_search_stats): queries in all-flat shortlist workgroups, computed when the
    // stats are read from the device count (last_flat_dev) and the launch shape; 0 when the search had no flat grouping
    const int *last_flat_dev = nullptr;
    long last_flat_nq = 0, last_flat_qpw = 0, last_flat_wgs = 0;
    hipEvent_t done_event = nullptr;  // recorded at the end of every search on its stream (stats wait on it)
    int last_orbit = 0;         // 1: the last search ran the mirror-orbit path
    OrbitIndex *orbit = nullptr; // mirror-orbit index (orbit.hip), null when not applicable
    KdTree *kd = nullptr;       // KD_SPLIT_STD tree: ties resolve in ANN's first-found order (null: lowest index)
    int bs = 1, split = KD_SPLIT_STD;
    int *h_fb_count = nullptr;  // pinned
};

// build the device index from fp32 rows already in HBM (takes ownership of d_rows); split = KD_SPLIT_STD builds
// ANN's kd-tree with bucket size bs for the tie order, TILER_SPLIT_INDEX_ORDER resolves ties to the lowest index
NNIndex *nn_index_create_dev(float *d_rows, int n, int d, int bs, int split, hipStream_t stream);
void nn_index_destroy(NNIndex *ix);
// release a SearchScratch's device buffers (an index's own, or a coalescer slot's)
void nn_scratch_free(SearchScratch &s, bool synced = false);
// the search nn_search_dev runs for nq queries of k: the small-batch scan (true), which touches nothing of the index
// but its read-only data and the scratch, or the shortlist path
bool nn_search_is_small(const NNIndex *ix, int nq, int k);

struct FtMaps {
    int32_t *tile = nullptr, *pal = nullptr;
    uint8_t *hm = nullptr, *vm = nullptr;
};

// k nearest neighbours of nq fp32 query rows in HBM; results [nq][k] in HBM; async on stream.
// If maps is non-null (k == 1) the FrameTiling tilemap items are written too.
// h_idx / h_err (host-visible, fine-grained pinned memory, or null): a small-batch scan (nn_search_is_small) also
// writes its final results there from the device, so the caller needs no copy back; any other search leaves them.
int nn_search_dev(NNIndex *ix, const float *d_q, int nq, int k, int *d_idx, float *d_err, const FtMaps *maps,
                  hipStream_t stream, bool rootbox_ready = false, bool orbit_prepared = false, int *h_idx = nullptr,
                  float *h_err = nullptr);

// batches of at most max_k1 queries (k = 1) / max_k8 (k <= 8) take the exhaustive small-batch scan; 0 disables it
void nn_set_scan_limits(int max_k1, int max_k8);
// test hook: every kd pruning check lists its query for the exact replay (results unchanged)
void nn_set_force_replay(int on);
void nn_set_shortlist_gate(int on);

// frame tiling: RGB tiles -> descriptors (fp32) -> search -> tilemap items
int nn_frame_tiling_dev(NNIndex *ix, const int32_t *d_rgb, int Q, int use_wavelets, int gamma, int *d_idx,
                        float *d_err, const FtMaps *maps, hipStream_t stream);

}  // namespace tiler

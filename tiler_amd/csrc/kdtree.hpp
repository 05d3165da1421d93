// kdtree.hpp -- the reference's ANN 1.1.2 kd-tree (ann_kdtree_create(..., bs, ANN_KD_STD), main.pas:3779,3961)
// over an HBM-resident dataset, kept for ONE purpose: reproducing which of several equal-distance candidates
// ANN returns (its first-found order, extern.pas:65-67 / main.pas:3830,4027), bit for bit.  The search itself
// stays the exact MFMA search of nn_search.hip / orbit.hip; this tree orders ties, checks ANN's box pruning
// along the winner's path and, where that check cannot vouch for the result, replays ANN's search exactly.
//
// Shape (kd_split: n_lo = n / 2, annMedianSplit): a node covering pidx positions [s, e) with e - s > bs splits
// at m = s + (e - s) / 2 into LO [s, m) and HI [m, e).  The shape is implicit; split positions m are unique,
// so internal nodes are indexed by m (1..n-1).  Leaves are buckets of <= bs consecutive positions.
#pragma once
#include "tiler_common.hpp"

namespace tiler {

// ANNsplitRule (extern.pas:21-28) plus this library's extension: no tree, ties to the lowest index
enum { KD_SPLIT_STD = 0, KD_SPLIT_INDEX_ORDER = 100 };  // = include/tiler_ann.h TILER_SPLIT_*

// Device view.  pos == nullptr: index order (the lowest candidate index wins a tie).
struct KdOrder {
    const int *pos = nullptr;               // [n] point -> leaf position
    const int *pidx = nullptr;              // [n] leaf position -> point
    const int *cd = nullptr;                // [n] cut dimension of internal node m
    const float *cv = nullptr;              // [n] cut value
    const float *lo = nullptr, *hi = nullptr;        // [n] cell bounds along cd (ANNkd_split::cd_bnds)
    const float *box_lo = nullptr, *box_hi = nullptr; // [dd] enclosing box of the dataset (annEnclRect)
    int n = 0, bs = 1, dd = 0;
};

struct KdTree {
    int n = 0, dd = 0, bs = 1;
    int *d_pos = nullptr, *d_pidx = nullptr, *d_cd = nullptr;
    float *d_cv = nullptr, *d_lo = nullptr, *d_hi = nullptr, *d_box = nullptr;  // d_box: [2][dd]
    KdOrder *d_view = nullptr;  // device copy of view(): what the search kernels get (one pointer)
    double build_ms = 0.0;
    int levels = 0;
    KdOrder view() const;
};

// Builds the tree of d_rows[n][dd] (fp32, HBM) exactly as ANN's kd_tree constructor does; synchronous.
KdTree *kd_tree_build(const float *d_rows, int n, int dd, int bs, hipStream_t stream);
void kd_tree_destroy(KdTree *t, bool synced = false);  // synced: the caller already synchronised the device
// leaf position of every point (host copy), for tests
int kd_tree_positions(const KdTree *t, int32_t *pos);

// After a search wrote idx/err [nq][k] (ascending, ties in kd order): check ANN's box pruning along every
// result's path; a query whose result the check cannot vouch for is searched again by an exact replay of
// annkSearch.  maps (k == 1): tilemap items are rewritten for replayed queries.
struct KdFixArgs {
    const float *rows, *q;
    int nq, k;
    int *idx;
    float *err;
    const int32_t *tr_tile = nullptr, *tr_pal = nullptr;
    const uint8_t *tr_attr = nullptr;
    int32_t *m_tile = nullptr, *m_pal = nullptr;
    uint8_t *m_hm = nullptr, *m_vm = nullptr;
    int *list = nullptr, *count = nullptr;  // [nq], [1]: queries sent to the replay (count zeroed by the caller)
    const float *rootbox = nullptr;         // [nq] annBoxDistance of every query (kd_root_boxes)
    const uint8_t *done = nullptr;          // [nq] or null: 1 = already checked (the pair pass), skip
    int force_replay = 0;                   // test hook (tiler_debug_force_replay): vouch for nothing
};
// rootbox[q] = annBoxDistance(q, box) for nq fp32 rows q[nq][dd] (queries whose descriptor kernel did not fuse it)
// annBoxDistance of every query to the root box; done[nq] / count (optional) are zeroed by the same launch
int kd_root_boxes(const KdTree *t, const float *d_q, int nq, float *rootbox, hipStream_t stream,
                  uint8_t *done = nullptr, int *count = nullptr);
int kd_verify_and_replay(const KdTree *t, const KdFixArgs &a, hipStream_t stream);
// the exact replay of the queries already listed in a.list / *a.count (the small-batch merge checks them itself)
int kd_replay_listed(const KdTree *t, const KdFixArgs &a, hipStream_t stream);
// annkPriSearch (ANN.dll 0x1800121a0, k = 1 as ann_kdtree_pri_search 0x180003ef0 calls it) replayed exactly for nq
// queries, one thread each: box-distance priority queue (ANNpr_queue, 1-based binary heap of at most n entries),
// leaf scans as annkSearch's, (1 + eps)^2 termination.  heap: kd_pri_heap_bytes(t, nq) of device scratch.
size_t kd_pri_heap_bytes(const KdTree *t, int nq);
// only (device flags [nq], or null = all): the queries to replay (kd_pri_resolve's fallbacks)
// (flag 2: the heap alone up to the first leaf holding one of kd_pri_resolve's targets, read from aux)
int kd_pri_search(const KdTree *t, const float *d_rows, const float *d_q, int nq, float eps, void *heap, int *d_idx,
                  float *d_err, hipStream_t stream, const uint8_t *only = nullptr, const void *aux = nullptr);
// eps = 0: the priority search's answer from annkSearch's (d_err0 = its distances) and the exact tie set (every point
// within that distance, then the entry keys of the points at the minimum); writes d_idx / d_err of the queries it
// decides and flag[q] = 1 for the others (to kd_pri_search).  aux: kd_pri_aux_bytes(nq) of device scratch.
size_t kd_pri_aux_bytes(int nq);
int kd_pri_resolve(const KdTree *t, const float *d_rows, const float *d_q, int nq, const float *d_err0, void *aux,
                   int *d_idx, float *d_err, uint8_t *flag, hipStream_t stream);

}  // namespace tiler

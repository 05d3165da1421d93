// orbit.hpp -- mirror-orbit FrameTiling search (gfx950): one MFMA pass scores all 4 H/V mirrors of a tile.
//
// The a6 search dataset (PrepareFrameTiling.DoPsyV, main.pas:3883-3919) holds every used tile in up to
// 4 orientations, emitted consecutively (hmir inner, vmir outer).  For the Haar PsyV descriptor
// (WaveletGS main.pas:2805-2840, the FrameTiling default `chkUseWL`) a mirrored tile's descriptor is an
// EXACT signed permutation of the unmirrored one (L = (a+b)*f and H = (a-b)*f are symmetric /
// antisymmetric in a, b bit for bit), so with S_m the signed permutation of mirror m and the isotypic
// decomposition of R^192 under {I, H, V, HV} (4 components of 48 dimensions each),
//     q . (S_m c) = sum_x chi_x(m) (P_x q) . (P_x c),   chi_x(m) = (-1)^popcount(x & m).
// The shortlist therefore runs one 192-deep MFMA contraction per (query, tile) instead of 4, keeping
// the 4 partial 48-d dots in separate accumulators; everything downstream stays exact.
// Grouping is data-driven and verified bit-for-bit on the device, so the path also serves the
// reference's plain `ann_kdtree_create` + `ann_kdtree_search` calls (extern.pas:63-67).
#pragma once
#include "nn_search.hpp"

namespace tiler {

// per-query statistics of the transformed query q' (scaled space)
struct OrbitStat {
    double n2;   // ||q||^2
    double hn;   // ||fp16(q')||
    double en;   // ||q' - fp16(q')||
    int flags;   // bit1: bad (non-finite / fp16 overflow) -> exhaustive scan
    int pad;
};

// ANN's visit order restricted to one orbit group's (<= 4) candidates: the kd-tree nodes that separate them
// (<= 3, their lowest common nodes) and, per slot pair (x < y), which node decides and whether x lies LO.  With
// it a tie between two members of one group costs 1 cached compare instead of a root-to-leaf walk.
struct GroupOrder {
    uint16_t cd[3];
    uint16_t pad;
    float cv[3];
    uint32_t pairs;  // 3 bits per pair index (0,1) (0,2) (0,3) (1,2) (1,3) (2,3): node (2 bits) | x-on-LO << 2
};

struct OrbitIndex {
    int G = 0, gblk = 0;          // tile groups (orbits of candidates) and 32-group blocks
    void *d_frag = nullptr;       // [gblk][12][64][8] fp16 MFMA A fragments of c' = U c_base
    void *d_rowh = nullptr;       // [G][192] fp16 c' row-major (rescore re-keying)
    float *d_seed = nullptr;      // [gblk][32] -||c||^2/2 in accumulator-row order (-inf padding)
    float *d_nc = nullptr;        // [G] ||c||^2 (scaled, fp32)
    int *d_member = nullptr;      // [G][4] candidate index of relative mirror slot m (H = 1, V = 2), -1 absent
    uint8_t *d_dup = nullptr;     // [G] bit m: slot m's row repeats a lower-index member's (symmetric tiles)
    uint8_t *d_rep = nullptr;     // [G] 2 bits per slot: the slot holding the lowest-index copy of its row
    GroupOrder *d_gorder = nullptr;  // [G] (kd tie order only)
    int *d_grp_of = nullptr;      // [n] candidate -> g * 4 + slot (kd tie order only; -1: not in a group)
    void *d_map = nullptr;        // OrbitMap
    float *d_base = nullptr;      // [ceil(G / 64)][48][64] float4: fp32 base row (member slot 0) of every group, float4
                                  // piece k of group g at [g / 64][k][g % 64] (zero padding); null when the compiled
                                  // mirror tables (orbitgen::MSRC / MNEG) do not match build_map (small-batch orbit scan)
    // mirror-symmetric groups first (orbit_build): blocks [0, red_end) may have isotypic blocks of c' that are zero
    // for every group in them (bit x of d_bmask[blk] clear), whose k-steps the shortlist skips; the rest are full
    int red_end = 0;
    int ksteps = 0;               // k-steps issued per query: 12 per full block, 3 per nonzero isotypic block below red_end
    uint8_t *d_bmask = nullptr;   // [red_end] union of the block's groups' nonzero isotypic blocks
    uint8_t *d_bmask0 = nullptr;  // [gblk] all 1 (block 0 only): the shortlist of flat query tiles
    double N = 0, Np = 0, Hp = 0, Ecp = 0;  // max ||c||, ||c'||, ||fp16(c')||, ||c' - fp16(c')||
    // per-call scratch
    void *qfrag = nullptr;        // [nqblk][12][64][8] fp16 q' (MFMA B fragments; the rescore re-keys from them)
    OrbitStat *qstat = nullptr;
    int *pair_cnt = nullptr, *pair_cand = nullptr;  // rescore -> pair pass hand-off
    size_t cap_q = 0;
    float *key = nullptr;
    int *id = nullptr;
    size_t cap_keys = 0;
    int *d_stats = nullptr;         // [2] expansion passes, candidates rescored (TILER_ORBIT_STATS=1)
    long long last_expansions = 0, last_rescored = 0;
    // the first query half's rescore and pair pass run on their own stream beside the second half's shortlist
    hipStream_t tail_stream = nullptr;
    hipEvent_t ev_half = nullptr, ev_tail = nullptr;
};

// generic tier-2 / tier-3 plumbing the orbit rescore feeds (owned by nn_search.hip)
struct OrbitTail {
    int *fb_list, *fb_count, *ex_list, *ex_count, fb_max;  // fb_max = nq: every tier-2 query has a slot
    float *thr;                   // [nq] tier-2 threshold T_b (bound-key domain, fp32 rounded up), set by the rescore
    unsigned long long *t2_best;  // [nq] per tier-2 slot: min (distance bits << 32 | kd_rank), ~0 until scored
    const int *flat_cnt;          // device [1] or null: queries >= *flat_cnt are flat tiles (only isotypic block 0 of
                                  // q' is nonzero); read by the shortlist itself, so no host round trip
    int *out_idx;
    float *out_err;
    const int32_t *tr_tile, *tr_pal;
    const uint8_t *tr_attr;
    int32_t *m_tile, *m_pal;
    uint8_t *m_hm, *m_vm;
    int *n_expand;                // optional device counter of block expansions
    const KdOrder *ko;            // tie order: ANN's kd-tree first-found (device view), nullptr = lowest index
    const float *kd_rootbox;      // [nq] (ko != nullptr): each query's annBoxDistance to the tree's box
    uint8_t *kd_done;             // [nq] the pair pass marks the queries whose winner it checked
    int *kd_list, *kd_count;      // queries whose winner ANN's pruning might have skipped -> exact replay
};

// 0: orbit index built (ix->orbit), 1: dataset has no exploitable mirror structure, -1: HIP error
int orbit_build(NNIndex *ix, hipStream_t stream);
void orbit_destroy(OrbitIndex *o, bool synced = false);
inline long long orbit_groups(const NNIndex *ix) { return ix->orbit ? ((const OrbitIndex *)ix->orbit)->G : 0; }
inline int orbit_ksteps(const NNIndex *ix) { return ix->orbit ? ((const OrbitIndex *)ix->orbit)->ksteps : 0; }
// rescore counters of the last search (TILER_ORBIT_STATS=1, else 0): 4-entry expansion passes, candidates rescored
void orbit_counters(const NNIndex *ix, long long *expansions, long long *rescored);
// k = 1 search of nq fp32 query rows: query prep, orbit shortlist, orbit rescore (tiers 2/3 by the caller);
// queries_prepared: orbit_ft_queries already wrote this call's fragments and statistics
int orbit_search(NNIndex *ix, const float *d_q, int nq, const OrbitTail &tail, hipStream_t stream,
                 bool queries_prepared = false);
int orbit_ensure_queries(OrbitIndex *o, int nq);
// tier 2 of an orbit search, for every query the rescore listed (device count, fixed grid, no host read): every
// orbit re-scored; each member whose mirror key reaches thr[q] gets its reference distance and ANN rank at once and
// an atomic minimum into t2_best[j]; then the winners are decoded and written (tail's outputs).  No candidate
// buffer, so no capacity to overflow: only non-finite / fp16-overflowing queries reach the exhaustive tier 3.
int orbit_tier2(NNIndex *ix, const float *d_q, const OrbitTail &tail, int nq, hipStream_t stream);
// FrameTiling queries in one kernel: RGB tiles -> Haar descriptors (qrows[Q][192] fp32) + q' fragments + stats
// (+ rootbox[Q] = annBoxDistance to box[2][192] when box != null)
// (perm: query i is tile perm[i] of d_rgb; null = identity)
int orbit_ft_queries(NNIndex *ix, const int32_t *d_rgb, int Q, int gamma, float *qrows, const float *box,
                     float *rootbox, hipStream_t stream, const int *perm = nullptr);

}  // namespace tiler

// prepare.hpp -- PrepareFrameTiling (main.pas:3791-3967) for one keyframe, on the device (internal interface).
#pragma once
#include "nn_search.hpp"

namespace tiler {

// scratch reused from keyframe to keyframe (kept with the global dataset's handle: no allocation, hence no
// device-wide hipFree synchronisation, between keyframes once the largest sizes have been seen)
struct PrepScratch {
    unsigned *bits = nullptr;      // [ceil(P*T/32)] distinct-item bitmap
    int *bcnt = nullptr;           // per-block counts / offsets (both compactions)
    int *total = nullptr;          // [2] device counts: distinct items, candidates
    int *keys = nullptr;           // [distinct] pal * T + tile, ascending
    float *qrows = nullptr;        // [distinct][64] the items' palette-index lines (UseOne's query)
    int *nn_idx = nullptr;         // [distinct][8]
    float *nn_err = nullptr;       // [distinct][8]
    uint8_t *near = nullptr;       // [P][P] Medium: near[p'][p] = corr(p', p) < tol * highest
    uint8_t *used = nullptr;       // [P][T][4]
    int32_t *tile_of = nullptr, *pal_of = nullptr;  // [cand] DoPsyV emission order
    uint8_t *attrs = nullptr, *flags = nullptr;     // [cand]
    int *h_total = nullptr;        // pinned [2]
    // recorded on the caller's stream after the last read of this scratch (the TRTo* map copies); the next prepare,
    // possibly on another stream, waits on it before it writes the scratch again
    hipEvent_t done = nullptr;
    size_t cap_bits = 0, cap_items = 0, cap_used = 0, cap_cand = 0, cap_near = 0, cap_blk = 0;
};
void prep_scratch_free(PrepScratch *s);

// The keyframe's search index (with its TRTo* maps) from its tilemap items: distinct (PalIdx, GlobalTileIndex)
// -> k = 8 preselection in the global dataset `global` (PrepareGlobalFT's handle, maps set) -> used[P][T][4]
// (UseOne: results of equal err after the first skipped; Fast: own palette, Medium: near[][], Slow: all) ->
// candidates in DoPsyV order -> descriptors -> index.  Synchronises `stream` once (the candidate count).
NNIndex *prepare_frame_tiling_dev(NNIndex *global, PrepScratch &s, const int32_t *d_item_tile,
                                  const int32_t *d_item_pal, long n_items, const uint8_t *d_palpix,
                                  const uint8_t *d_thm, const uint8_t *d_tvm, int T, const int32_t *d_palettes, int P,
                                  int quality, const uint8_t *h_near, int use_wavelets, int gamma, hipStream_t stream,
                                  long *n_distinct, long *n_cand);

}  // namespace tiler

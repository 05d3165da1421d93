// smooth.hpp -- Smooth (DoTemporalSmoothing main.pas:4071-4119) on gfx950 (internal interface).
#pragma once
#include "tiler_common.hpp"

namespace tiler {
int smooth_keyframe_host(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                         uint8_t *smoothed, int T, const uint8_t *palpix, int P, const int32_t *palettes,
                         double strength);
// all pointers in HBM; asynchronous on stream
int smooth_keyframe_dev(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                        uint8_t *sm, const uint8_t *palpix, const int32_t *palettes, double strength,
                        hipStream_t stream);
}  // namespace tiler

// keyframes.hpp -- Load-step keyframe detection (main.pas:811-828, 1099-1146, 1465-1492) on gfx950 (internal).
#pragma once
#include "tiler_common.hpp"

namespace tiler {
// frames [F][tm_h*tm_w][64] int32 0x00BBGGRR; corr[F-1] (host) = ComputeInterFrameCorrelation(i-1, i)
int interframe_corr_host(const int32_t *rgb, int F, int tm_w, int tm_h, double *corr);
// frames in HBM (16-byte aligned); corr is a HOST buffer; synchronises `stream`
int interframe_corr_dev(const int32_t *d_rgb, int F, int tm_w, int tm_h, double *corr, hipStream_t stream);
// keyframe index per frame; returns the keyframe count (or -1)
int find_keyframes(const double *corr, int F, int tile_map_size, int32_t *kf_of_frame);
}  // namespace tiler

// palette.hpp -- palette generation of the Dither step (QuantizePalette / DLv3, FinishQuantizePalette).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tiler {

// QuantizePalette with DLv3 for P (keyframe, palette) pairs: tiles rgb[n][64] 0x00BBGGRR, pal_of[n] (pair index,
// others skipped), active[n] or null -> pal_out[P][palsize] (CompareCMULHS order), use_count[P], hist[P] (null ok:
// the DLv3 colour-table sizes).  Host outputs.
void dl3_debug(int list_cap);  // tiler_debug_dl3
int quantize_palettes_dev(long n_tiles, const int32_t *d_rgb, const int32_t *d_pal_of, const uint8_t *d_active, int P,
                          int palsize, int bpc, int32_t *pal_out, int32_t *use_count, int32_t *hist, hipStream_t stream);
int quantize_palettes_host(long n_tiles, const int32_t *rgb, const int32_t *pal_of, const uint8_t *active, int P,
                           int palsize, int bpc, int32_t *pal_out, int32_t *use_count, int32_t *hist);
// CMPal.Sort(@CompareCMULHS) of one palette in place
void sort_palette_cmulhs(int32_t *pal, int n);
// FinishQuantizePalette's order: lut[old palette] = new index (kmodes.pas QuickSort, use count descending)
void finish_quantize_order(const int32_t *use_count, int P, int32_t *lut);

}  // namespace tiler

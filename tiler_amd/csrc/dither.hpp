// dither.hpp -- FinishDitherTiles per-tile work (Thomas Knoll DitherTile + PrepareTileMirrors) on gfx950 (internal).
#pragma once
#include "tiler_common.hpp"

namespace tiler {
int dither_tiles_tk_host(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int n_palettes,
                         int palsize, uint8_t *palpix, uint8_t *hm, uint8_t *vm);
// all pointers in HBM; asynchronous on stream
int dither_tiles_tk_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes,
                        int n_palettes, int palsize, uint8_t *d_palpix, uint8_t *d_hm, uint8_t *d_vm,
                        hipStream_t stream);
}  // namespace tiler

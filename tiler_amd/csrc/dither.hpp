// dither.hpp -- FinishDitherTiles per-tile work (DitherTile with Thomas Knoll or Yliluoma mixing + PrepareTileMirrors)
// on gfx950 (internal).  mixed = 0: Thomas Knoll (the reference default); 1..64: Yliluoma, Y2MixedColors = mixed.
#pragma once
#include "tiler_common.hpp"

namespace tiler {
int dither_tiles_host(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int n_palettes,
                      int palsize, int mixed, uint8_t *palpix, uint8_t *hm, uint8_t *vm);
// all pointers in HBM; asynchronous on stream
int dither_tiles_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes, int n_palettes,
                     int palsize, int mixed, uint8_t *d_palpix, uint8_t *d_hm, uint8_t *d_vm, hipStream_t stream);
}  // namespace tiler

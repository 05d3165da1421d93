// psyv.hpp -- descriptor kernel interface (internal).
#pragma once
#include "tiler_common.hpp"

namespace tiler {

enum { PSYV_FROM_PAL = 1, PSYV_WAVELETS = 2, PSYV_LAB = 4, PSYV_QWEIGHT = 8, PSYV_HMIRROR = 16, PSYV_VMIRROR = 32 };

struct PsyvArgs {
    long n = 0;
    const int32_t *rgb = nullptr;       // [n][64]
    const uint8_t *palpix = nullptr;    // [T][64]
    const int32_t *tile_of = nullptr;   // [n] or null (identity)
    const int32_t *palettes = nullptr;  // [P][16]
    const int32_t *pal_of = nullptr;    // [n] or null (palette 0)
    const uint8_t *flags_per = nullptr; // [n] or null
    bool flags_per_mirrors_only = false; // flags_per holds only PSYV_HMIRROR / PSYV_VMIRROR bits (caller's promise)
    int flags = 0;
    int gamma = -1;
    double *out64 = nullptr;            // [n][192]
    float *out32 = nullptr;             // [n][192]
    // optional (RGB Haar query path only): annBoxDistance of the fp32 descriptor to box[2][192] (a kd-tree's
    // enclosing box, kdtree.hpp) -> rootbox[n], fused so the FrameTiling search's pruning check needs no re-read
    const float *box = nullptr;
    float *rootbox = nullptr;
    // optional (RGB Haar query path only): descriptor i is made of tile rgb[perm[i]] (FrameTiling's flat grouping)
    const int *perm = nullptr;
    // filled by launch_psyv from the shared LUTs
    const double *gamma_lut = nullptr, *dct_lut = nullptr, *qmul = nullptr, *ratio = nullptr, *lab_lin = nullptr;
    double haar_f = 0, u_mul = 0, v_mul = 0;
};

int launch_psyv(PsyvArgs args, hipStream_t stream);

}  // namespace tiler

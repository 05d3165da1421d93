// kmeans.hpp -- the Dither step's k-means (PrepareDitherTiles' yakmo call, main.pas:2125-2133), kmeans.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tiler {

// X [n][d] fp64 in HBM (d <= 192) -> labels [n] (device), centroids [k][d] (device), *iterations (assignments run)
int kmeans_dev(const double *d_X, long n, int d, int k, int max_iter, uint32_t seed, int32_t *d_labels, double *d_cent,
               int *iterations, hipStream_t stream);

// PrepareDitherTiles for one keyframe: LAB (+ wavelet) descriptors of n_tiles RGB tiles -> k-means with k = P
int prepare_dither_dev(long n_tiles, const int32_t *d_rgb, int P, int gamma, int use_wavelets, int max_iter,
                       uint32_t seed, int32_t *d_labels, double *d_cent, int *iterations, hipStream_t stream);

}  // namespace tiler

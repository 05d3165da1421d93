// kmodes.hpp -- K-Modes (TKModes, kmodes.pas) on gfx950 (internal interface).
#pragma once
#include "tiler_common.hpp"

namespace tiler {
int kmodes_compute_host(const uint8_t *X, int n, int nattr, int k, int start_point, int n_modalities,
                        int32_t *labels, uint8_t *centroids, int *n_iter, uint64_t *cost);
int kmodes_medoids_host(const uint8_t *X, int n, const int32_t *labels, const uint8_t *centroids, int k,
                        int32_t *medoid, int32_t *counts);
// X [n][80] in HBM (16-byte aligned), labels [n] / centroids [k][80] in HBM; returns 0 / -1
int kmodes_compute_dev(const uint8_t *d_X, int n, int k, int start_point, int n_modalities, int32_t *d_labels,
                       uint8_t *d_centroids, int *n_iter, uint64_t *cost, hipStream_t st);
}  // namespace tiler

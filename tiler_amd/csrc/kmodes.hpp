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
// all GlobalTiling palette bins at once: X [N][80] with bin b = rows [boff[b], boff[b+1]); k / start per bin;
// labels bin-local, centroids [sum k][80] in bin order; n_iter / cost per bin (host arrays).  0 / -1
int kmodes_batch_dev(const uint8_t *d_X, const int32_t *h_boff, int nb, const int32_t *h_k, const int32_t *h_start,
                     int n_modalities, int32_t *d_labels, uint8_t *d_centroids, int32_t *h_iter, uint64_t *h_cost,
                     hipStream_t st);
int kmodes_batch_host(const uint8_t *X, const int32_t *boff, int nb, const int32_t *k, const int32_t *start,
                      int n_modalities, int32_t *labels, uint8_t *centroids, int32_t *n_iter, uint64_t *cost);
// the last batch's assignment (point, centroid) pairs and its dependent chunk steps
void kmodes_last_stats(long long *pairs, long long *steps);
// test hook: the persistent farthest-first's barriers give up at once, so the host's recovery path runs
void kmodes_force_ff_fallback(int on);
int kmodes_medoids_batch_host(const uint8_t *X, const int32_t *boff, int nb, const int32_t *k, const int32_t *labels,
                              const uint8_t *centroids, int32_t *medoid, int32_t *counts);
}  // namespace tiler

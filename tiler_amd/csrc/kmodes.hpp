// kmodes.hpp -- K-Modes (TKModes, kmodes.pas) on gfx950 (internal interface).
#pragma once
#include "tiler_common.hpp"

namespace tiler {
int kmodes_compute_host(const uint8_t *X, int n, int nattr, int k, int start_point, int n_modalities,
                        int32_t *labels, uint8_t *centroids, int *n_iter, uint64_t *cost);
}

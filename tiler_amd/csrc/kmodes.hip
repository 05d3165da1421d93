#include "kmodes.hpp"
namespace tiler {
int kmodes_compute_host(const uint8_t *, int, int, int, int, int, int32_t *, uint8_t *, int *, uint64_t *) {
    set_error("kmodes: not implemented yet");
    return -1;
}
}  // namespace tiler

#include "smooth.hpp"
namespace tiler {
int smooth_keyframe_host(int, int, int32_t *, int32_t *, int32_t *, uint8_t *, uint8_t *, uint8_t *, int,
                         const uint8_t *, int, const int32_t *, double) {
    set_error("smooth: not implemented yet");
    return -1;
}
}  // namespace tiler

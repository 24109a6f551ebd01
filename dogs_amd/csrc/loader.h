// loader.h -- pinned image ring + u8 -> float CHW conversion (loader.hip; C ABI in include/dogs_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dogs_hip.h"

namespace gs {
// read_image's float conversion of a u8 HWC image (C = 1, 3 or 4) into CHW (composite: RGBA -> 3 channels over
// black, read_image's num_channels == 4)
void launch_u8_to_chw(const uint8_t* in, int H, int W, int C, int composite, float* out, hipStream_t s);
}  // namespace gs

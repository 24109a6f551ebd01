// export.h -- GPU packing of the reference's export formats (export.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {
// keys[i] = order-preserving bits of -exp(s0 + s1 + s2) / (1 + exp(opacity_i)), vals[i] = i
void launch_splat_keys(uint32_t N, const float* scaling, const float* opacity, uint32_t* keys, uint32_t* vals,
                       hipStream_t s);
// out[32 r ..] = the .splat record of Gaussian order[r]
void launch_splat_pack(uint32_t N, const uint32_t* order, const float* xyz, const float* scaling,
                       const float* opacity, const float* rot, const float* f_dc, uint8_t* out, hipStream_t s);
// out[27 i ..] = the save_ply vertex record of Gaussian i
void launch_ply_pack(uint32_t N, const float* xyz, const float* f_dc, uint8_t* out, hipStream_t s);
}  // namespace gs

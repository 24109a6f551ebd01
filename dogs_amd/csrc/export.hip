// export.hip -- GPU packing of the trained Gaussians into the reference's export formats:
//
// k_splat_keys/k_splat_pack  GaussianSplatModel.save_splat (gaussian_splat_model.py:666-708): 32-B records
//                            (position f32x3, exp(scale) f32x3, RGBA u8, normalised quaternion u8x4) in ascending
//                            order of -exp(s0 + s1 + s2) / (1 + exp(opacity)).  The reference builds them one
//                            Gaussian at a time in a Python loop; here one stable radix sort and one pass.
// k_ply_pack                 GaussianSplatModel.save_ply (gaussian_splat_model.py:616-640): 27-B vertex records
//                            (x y z f32, nx ny nz = 0, red green blue u8 of the degree-0 SH colour).
// Arithmetic follows the reference's numpy/torch float32 expressions op by op (export_oracle.py restates them).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include "export.h"

namespace gs {

namespace {

constexpr float SH_C0F = 0.28209479177387814f;  // sh_utils.py:26 (the Python float meets float32 tensors)

// order-preserving map of a float to u32 (ascending floats -> ascending keys)
__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(256) k_splat_keys(uint32_t N, const float* __restrict__ scaling,
                                                    const float* __restrict__ opacity, uint32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= N) return;
    const float* s = scaling + 3 * (size_t)i;
    // -np.exp(scale[:, 0] + scale[:, 1] + scale[:, 2]) / (1 + np.exp(opacity[:, 0]))
    const float v = -expf((s[0] + s[1]) + s[2]) / (1.0f + expf(opacity[i]));
    keys[i] = fkey(v);
    vals[i] = i;
}

__device__ __forceinline__ uint8_t u8_trunc_clip(float v) {  // .clip(0, 255).astype(np.uint8)
    v = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
    return (uint8_t)(int)v;
}

__global__ void __launch_bounds__(256) k_splat_pack(uint32_t N, const uint32_t* __restrict__ order,
                                                    const float* __restrict__ xyz, const float* __restrict__ scaling,
                                                    const float* __restrict__ opacity, const float* __restrict__ rot,
                                                    const float* __restrict__ f_dc, uint8_t* __restrict__ out) {
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;
    if (r >= N) return;
    const uint32_t i = order[r];
    float rec[6];
    for (int c = 0; c < 3; c++) rec[c] = xyz[3 * (size_t)i + c];
    for (int c = 0; c < 3; c++) rec[3 + c] = expf(scaling[3 * (size_t)i + c]);
    uint8_t b[8];
    for (int c = 0; c < 3; c++) b[c] = u8_trunc_clip((0.5f + SH_C0F * f_dc[3 * (size_t)i + c]) * 255.0f);
    b[3] = u8_trunc_clip((1.0f / (1.0f + expf(-opacity[i]))) * 255.0f);
    const float* q = rot + 4 * (size_t)i;
    const float nrm = sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
    for (int c = 0; c < 4; c++) b[4 + c] = u8_trunc_clip((q[c] / nrm) * 128.0f + 128.0f);
    uint32_t w[8];
    for (int c = 0; c < 6; c++) w[c] = __float_as_uint(rec[c]);
    w[6] = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    w[7] = (uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24);
    uint4* o = reinterpret_cast<uint4*>(out + 32 * (size_t)r);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ void __launch_bounds__(256) k_ply_pack(uint32_t N, const float* __restrict__ xyz,
                                                  const float* __restrict__ f_dc, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= N) return;
    uint8_t rec[27];
    float v[6] = {xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1], xyz[3 * (size_t)i + 2], 0.0f, 0.0f, 0.0f};
    memcpy(rec, v, 24);
    for (int c = 0; c < 3; c++) {
        // torch: clamp_min(C0 * dc + 0.5, 0) -> numpy * 255 -> float32 attribute -> u1 field (C cast: values past
        // 255 wrap as the x86 float -> int -> byte conversion does)
        float x = fmaxf(SH_C0F * f_dc[3 * (size_t)i + c] + 0.5f, 0.0f) * 255.0f;
        rec[24 + c] = (uint8_t)(int)x;
    }
    uint8_t* o = out + 27 * (size_t)i;
    for (int k = 0; k < 27; k++) o[k] = rec[k];
}

}  // namespace

void launch_splat_keys(uint32_t N, const float* scaling, const float* opacity, uint32_t* keys, uint32_t* vals,
                       hipStream_t s) {
    if (N) k_splat_keys<<<(N + 255) / 256, 256, 0, s>>>(N, scaling, opacity, keys, vals);
}
void launch_splat_pack(uint32_t N, const uint32_t* order, const float* xyz, const float* scaling,
                       const float* opacity, const float* rot, const float* f_dc, uint8_t* out, hipStream_t s) {
    if (N) k_splat_pack<<<(N + 255) / 256, 256, 0, s>>>(N, order, xyz, scaling, opacity, rot, f_dc, out);
}
void launch_ply_pack(uint32_t N, const float* xyz, const float* f_dc, uint8_t* out, hipStream_t s) {
    if (N) k_ply_pack<<<(N + 255) / 256, 256, 0, s>>>(N, xyz, f_dc, out);
}

}  // namespace gs

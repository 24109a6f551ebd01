// aux_kernels.h -- launchers of fused SSIM, sparse Adam and simple-knn (aux_kernels.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gs {
void launch_ssim_fwd(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2, float* map,
                     float* dmu1, float* ds1, float* ds12, hipStream_t s);
void launch_ssim_bwd(int B, int CH, int H, int W, const float* img1, const float* img2, const float* dL,
                     const float* dmu1, const float* ds1, const float* ds12, float* dimg1, hipStream_t s,
                     float dl_value = 0.0f);
// fused_ssim's mean in one pass (MEAN strips: no map; part [ssim_mean_parts()] per-wave map sums, then *mean = their
// total / numel in a fixed order) and its backward from the mean's gradient (device scalar, dL/dmap = *dl_mean / numel)
void launch_ssim_mean(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                      float* dmu1, float* ds1, float* ds12, float* part, float* mean, hipStream_t s);
void launch_ssim_mean_bwd(int B, int CH, int H, int W, const float* img1, const float* img2, const float* dl_mean,
                          const float* dmu1, const float* ds1, const float* ds12, float* dimg1, hipStream_t s);
uint32_t ssim_mean_parts(int B, int CH, int H, int W);
// *out = sum(part[0..n)) / denom in a fixed order (one block)
void launch_mean_parts(const float* part, uint32_t n, uint32_t denom, float* out, hipStream_t s);
// the native training step's variants: clamp(0, 1) of the raw render, the L1 term and the SSIM mean folded into the
// forward (part: ssim_waves() L1 partials, then as many map partials; no map written), and the clamp / L1 backward
// folded into the backward (d_raw: dL/d raw render; l1_scale = dL/dL1 / n)
uint32_t ssim_waves(int planes, int H, int W);
// mask (optional, [3,H,W]): the appearance mask -- the L1 partials are of |clamped * mask - gt| and a third set of
// ssim_waves() partials holds sum (mask - 1)^2
void launch_ssim_fwd_fused(int H, int W, float C1, float C2, const float* raw, const float* gt, float* clamped,
                           float* dmu1, float* ds1, float* ds12, float* part, hipStream_t s,
                           const float* mask = nullptr);
// The step's loss from the partial sums (optim.hip k_loss_final's outputs: loss[0] L1, [1] SSIM mean, [2] mean
// prod(scaling), [3] mean (mask - 1)^2 when p_mreg); launch_ssim_bwd_fused runs it as block 0 of its launch when given
// one.
struct LossFinal {
    const float *p_l1, *p_ssim, *p_sc;
    uint32_t n_l1, n_ssim, n_sc, n_img, P;
    float* loss;
    const float* p_mreg;
    uint32_t n_mreg;
};
// mask (optional): dL/dclamped of the L1 term is l1_scale sgn(clamped * mask - gt) * mask, and dmask receives
// l1_scale sgn(clamped * mask - gt) * clamped + mreg_scale (mask - 1)
void launch_ssim_bwd_fused(int H, int W, const float* clamped, const float* gt, const float* raw, float dl_value,
                           float l1_scale, const float* dmu1, const float* ds1, const float* ds12, float* d_raw,
                           hipStream_t s, const LossFinal* lf = nullptr, const float* mask = nullptr,
                           float* dmask = nullptr, float mreg_scale = 0.0f);
void launch_adam(float* param, const float* grad, float* m, float* v, const bool* visible, float lr, float b1, float b2,
                 float eps, uint32_t N, uint32_t M, hipStream_t s);
size_t knn_temp_bytes(int P);
void launch_knn(int P, const float* pts, float* out, void* temp, hipStream_t s);
}  // namespace gs

// aux_kernels.hip -- the satellite kernels that ship in the same extension as the rasterizer:
//   fused SSIM forward/backward  (fused-ssim/ssim.cu:187-366 semantics)
//   sparse Adam                  (cuda_rasterizer/adam.cu:10-38)
//   simple-knn distCUDA2         (simple-knn/simple_knn.cu:45-221)
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>
#include "aux_kernels.h"
#include "sortscan.h"

namespace gs {

// ------------------------------------------------------------------------------------------------
// fused SSIM (ssim.cu:187-444 semantics).  One wave per strip of 54 output columns x 32 output rows of one
// plane: the 64 lanes hold 54 + 10 halo columns, so the horizontal 11-tap pass is a chain of DPP wave_shl:1 moves
// (lane i <- lane i+1) with no LDS at all, and the vertical pass runs over a ring of the last 11 rows' horizontal
// moments in registers (the 11-row loop is unrolled so every ring slot is a compile-time register).  Products and
// fma order per moment are the reference's (x taps 0..10, then y taps 0..10).  Rows are read SSIM_PF ahead of use.
// (The first version staged 42x42 halo tiles and the x-pass moments in LDS: forward 94-102 us, backward 80 us at
// 1080p x 3; this one: 94 and 60.)
// ------------------------------------------------------------------------------------------------
constexpr int SSW_OUT = 54;   // output columns per wave
#ifndef DG_SSW_ROWS
#define DG_SSW_ROWS 32
#endif
constexpr int SSW_ROWS = DG_SSW_ROWS;  // output rows per wave
constexpr int SSW_IN = SSW_ROWS + 10;
#ifndef DG_SSIM_PF
#define DG_SSIM_PF 2
#endif
constexpr int SSIM_PF = DG_SSIM_PF;   // input rows loaded ahead of use (a register queue of SSIM_PF rows)
constexpr float GW[11] = {0.001028380123898387f, 0.0075987582094967365f, 0.036000773310661316f,
                          0.10936068743467331f, 0.21300552785396576f, 0.26601171493530273f,
                          0.21300552785396576f, 0.10936068743467331f, 0.036000773310661316f,
                          0.0075987582094967365f, 0.001028380123898387f};

__device__ __forceinline__ float wave_shl1(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x130, 0xf, 0xf, false));
}
// sum_k GW[k] * x(lane + k), k = 0..10.
// Default: Horner form over the lanes -- acc <- shl1(acc) + GW[k] x from k = 10 down to 0 -- where the DPP shift folds
// into the add (v_add_f32_dpp) and the window is symmetric, so the products are the six GW[k] x of k <= 5: 16 VALU per
// convolution instead of 21 (10 DPP moves + 11 fmas).  The sum runs k = 10 .. 0 with rounded products (a few ulp from
// the reference's k = 0 .. 10 order, inside the 1e-5 parity bar).  DG_SSIM_TAPFMA: the tap-order fma chain.
__device__ __forceinline__ float wave_shl1_add(float acc, float t) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(acc), 0x130, 0xf, 0xf, false)) + t;
}
__device__ __forceinline__ float hconv11(float x) {
#ifdef DG_SSIM_TAPFMA
    float acc = fmaf(GW[0], x, 0.0f);
#pragma unroll
    for (int k = 1; k < 11; k++) {
        x = wave_shl1(x);
        acc = fmaf(GW[k], x, acc);
    }
    return acc;
#else
    float t[6];
#pragma unroll
    for (int k = 0; k < 6; k++) t[k] = GW[k] * x;
    float acc = t[0];                               // k = 10 (GW[10] = GW[0])
#pragma unroll
    for (int k = 9; k >= 0; k--) acc = wave_shl1_add(acc, t[k <= 5 ? k : 10 - k]);
    return acc;
#endif
}

// Q window sums at once with their Horner chains interleaved step by step: a DPP read of a VGPR needs two wait
// states after the VALU write of it, and one chain alone puts an s_nop before almost every v_add_f32_dpp (503 of 508
// in the forward); with Q >= 3 chains the other chains' adds fill them.  Same arithmetic per sum as hconv11.
template <int Q>
__device__ __forceinline__ void hconv11_n(const float (&x)[Q], float (&out)[Q]) {
#if defined(DG_SSIM_TAPFMA) || defined(DG_SSIM_CHAIN1)  // A/B: one sum at a time
#pragma unroll
    for (int q = 0; q < Q; q++) out[q] = hconv11(x[q]);
#else
    float t[Q][6];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
        for (int k = 0; k < 6; k++) t[q][k] = GW[k] * x[q];
#pragma unroll
    for (int q = 0; q < Q; q++) out[q] = t[q][0];
#pragma unroll
    for (int k = 9; k >= 0; k--)
#pragma unroll
        for (int q = 0; q < Q; q++) out[q] = wave_shl1_add(out[q], t[q][k <= 5 ? k : 10 - k]);
#endif
}

struct StripPos { int x, y0, plane; bool valid; };
__device__ __forceinline__ StripPos strip_of(int H, int W, int planes, uint32_t skip_blocks = 0) {
    const int sxn = (W + SSW_OUT - 1) / SSW_OUT, syn = (H + SSW_ROWS - 1) / SSW_ROWS;
    const int wid = (int)(blockIdx.x - skip_blocks) * 4 + (threadIdx.x >> 6);
    StripPos p;
    p.valid = wid < sxn * syn * planes;
    const int sx = wid % sxn, sy = (wid / sxn) % syn;
    p.plane = wid / (sxn * syn);
    p.x = sx * SSW_OUT - 5 + (threadIdx.x & 63);
    p.y0 = sy * SSW_ROWS;
    return p;
}

// torch.clamp(x, 0, 1), NaN kept (optim.hip clamp01)
__device__ __forceinline__ float clamp01f(float x) { return x != x ? x : fminf(fmaxf(x, 0.f), 1.f); }

// FUSED (the native training step): img1 is the raw render, read through clamp(0, 1); the clamped image goes to
// out_img, and each wave writes its partial sums of |clamped - gt| and of the map (part[wave], part[nwaves + wave])
// instead of the map itself -- render()'s clamp, the L1 term and the SSIM mean in the same pass.
// MASK (with FUSED): the appearance mask multiplies the clamped render inside the L1 term (|clamped * mask - gt|), and a
// third set of per-wave partials holds sum (mask - 1)^2 (gaussian_trainer.py:392-401)
// MEAN (the drop-in fused_ssim(...) = FusedSSIMMap(...).mean()): no clamp, no map written, each wave writes its partial
// sum of the map to part[wave] (the FUSED map partials' arithmetic: the same per-wave values), k_mean_parts totals them.
template <bool TRAIN, bool FUSED = false, bool MASK = false, bool MEAN = false>
__global__ void __launch_bounds__(256) k_ssim_fwd_strip(int H, int W, int planes, float C1, float C2,
                                                        const float* __restrict__ img1, const float* __restrict__ img2,
                                                        float* __restrict__ map, float* __restrict__ dmu1,
                                                        float* __restrict__ ds1, float* __restrict__ ds12,
                                                        float* __restrict__ out_img = nullptr,
                                                        float* __restrict__ part = nullptr,
                                                        const float* __restrict__ mask = nullptr) {
    const StripPos sp = strip_of(H, W, planes);
    if (!sp.valid) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const size_t plane = (size_t)sp.plane * H * W;
    const float* a = img1 + plane;
    const float* b = img2 + plane;
    const bool colok = sp.x >= 0 && sp.x < W;
    // the lane's window covers columns x .. x+10: its output is column x+5
    const int ox = sp.x + 5;
    const bool out_col = lane < SSW_OUT && ox < W;
    auto lda = [&](int row) -> float {
        if (!(colok && row >= 0 && row < H)) return 0.0f;
        const float x = a[(size_t)row * W + sp.x];
        return FUSED ? clamp01f(x) : x;
    };
    auto ldb = [&](int row) -> float {
        return (colok && row >= 0 && row < H) ? b[(size_t)row * W + sp.x] : 0.0f;
    };
    float acc_l1 = 0.0f, acc_map = 0.0f, acc_mreg = 0.0f;
    float ring[11][5];
    // FUSED: the clamped image and the L1 term as the input rows arrive -- lanes 5..58 hold the strip's output columns
    const bool own_col = FUSED && lane >= 5 && lane < 5 + SSW_OUT && colok;
    float qa[SSIM_PF], qb[SSIM_PF];
#pragma unroll
    for (int p = 0; p < SSIM_PF; p++) {
        qa[p] = lda(sp.y0 - 5 + p);
        qb[p] = ldb(sp.y0 - 5 + p);
    }
    for (int base = 0; base < SSW_IN; base += 11) {
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const int rr = base + j;
            if (rr < SSW_IN) {
                const float u = qa[0], v = qb[0];
#pragma unroll
                for (int p = 0; p + 1 < SSIM_PF; p++) {
                    qa[p] = qa[p + 1];
                    qb[p] = qb[p + 1];
                }
                qa[SSIM_PF - 1] = lda(sp.y0 - 5 + rr + SSIM_PF);
                qb[SSIM_PF - 1] = ldb(sp.y0 - 5 + rr + SSIM_PF);
                if (FUSED) {
                    const int row = sp.y0 - 5 + rr;  // one of the strip's output rows
                    if (own_col && row >= sp.y0 && row < sp.y0 + SSW_ROWS && row < H) {
                        const size_t gi = plane + (size_t)row * W + sp.x;
                        out_img[gi] = u;
                        if (MASK) {
                            const float mk = mask[gi], dm = mk - 1.0f;
                            acc_l1 += fabsf(u * mk - v);
                            acc_mreg += dm * dm;
                        } else {
                            acc_l1 += fabsf(u - v);
                        }
                    }
                }
                {
                    const float xs[5] = {u, u * u, v, v * v, u * v};
                    hconv11_n<5>(xs, ring[j]);
                }
                const int y = sp.y0 + rr - 10;
                if (rr >= 10 && y < H) {
                    float m[5] = {0, 0, 0, 0, 0};
#pragma unroll
                    for (int k = 0; k < 11; k++) {
#pragma unroll
                        for (int q = 0; q < 5; q++) m[q] = fmaf(GW[k], ring[(j + 1 + k) % 11][q], m[q]);
                    }
                    if (out_col) {
                        const float mu1 = m[0], mu2 = m[2];
                        const float sigma1_sq = fmaf(-mu1, mu1, m[1]);
                        const float sigma2_sq = fmaf(-mu2, mu2, m[3]);
                        const float sigma12 = fmaf(-mu1, mu2, m[4]);
                        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
                        const float Cc = fmaf(2.0f, mu1_mu2, C1);
                        const float D = fmaf(2.0f, sigma12, C2);
                        const float A = (mu1_sq + mu2_sq) + C1;
                        const float B = (sigma1_sq + sigma2_sq) + C2;
                        const size_t gi = plane + (size_t)y * W + ox;
#ifndef DG_SSIM_IEEEDIV  // reciprocals of the three denominators instead of seven IEEE divisions: forward 97 -> 81 us
                         // at 1080p x 3, within the 1e-5 parity bar (test_fused_ssim_matches_oracle)
                        const float rAB = __builtin_amdgcn_rcpf(A * B), rAAB = __builtin_amdgcn_rcpf(A * A * B),
                                    rABB = __builtin_amdgcn_rcpf(A * B * B);
                        if (FUSED || MEAN) {
                            acc_map += (Cc * D) * rAB;
                        } else {
                            map[gi] = (Cc * D) * rAB;
                        }
                        if (TRAIN) {
                            dmu1[gi] = ((mu2 * 2.0f * D) * rAB - (mu2 * 2.0f * Cc) * rAB - (mu1 * 2.0f * Cc * D) * rAAB +
                                        (mu1 * 2.0f * Cc * D) * rABB);
                            ds1[gi] = ((-Cc * D) * rABB);
                            ds12[gi] = ((2 * Cc) * rAB);
                        }
#else
                        if (FUSED || MEAN) acc_map += (Cc * D) / (A * B);
                        else map[gi] = (Cc * D) / (A * B);
                        if (TRAIN) {
                            dmu1[gi] = ((mu2 * 2.0f * D) / (A * B) - (mu2 * 2.0f * Cc) / (A * B) -
                                        (mu1 * 2.0f * Cc * D) / (A * A * B) + (mu1 * 2.0f * Cc * D) / (A * B * B));
                            ds1[gi] = ((-Cc * D) / (A * B * B));
                            ds12[gi] = ((2 * Cc) / (A * B));
                        }
#endif
                    }
                }
            }
        }
    }
    if (FUSED) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            acc_l1 += __shfl_xor(acc_l1, o);
            acc_map += __shfl_xor(acc_map, o);
            if (MASK) acc_mreg += __shfl_xor(acc_mreg, o);
        }
        if (lane == 0) {
            const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
            const int nw = ((W + SSW_OUT - 1) / SSW_OUT) * ((H + SSW_ROWS - 1) / SSW_ROWS) * planes;
            part[wid] = acc_l1;
            part[nw + wid] = acc_map;
            if (MASK) part[2 * nw + wid] = acc_mreg;
        }
    } else if (MEAN) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc_map += __shfl_xor(acc_map, o);
        if (lane == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc_map;
    }
}

// *out = (sum of part[0..n)) / denom in loss_final_block's order (strided per thread, the wave sums, then (w0 + w1) +
// (w2 + w3)): over the MEAN partials the SSIM mean equals the native step's loss[1] bit for bit.  One 256-thread block.
__global__ void __launch_bounds__(256) k_mean_parts(const float* __restrict__ part, uint32_t n, uint32_t denom,
                                                    float* __restrict__ out) {
    __shared__ float s_w[4];
    float acc = 0.0f;
    for (uint32_t i = threadIdx.x; i < n; i += 256) acc += part[i];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = ((s_w[0] + s_w[1]) + (s_w[2] + s_w[3])) / (float)denom;
}

// The step's loss (k_loss_final's arithmetic, 256 threads): each total strided per thread, then the 4 wave sums in order.
// loss[3]: mean (mask - 1)^2 from p_mreg, 0 without a mask.
__device__ __forceinline__ void loss_final_block(const LossFinal& f) {
    __shared__ float s_w[4][4];
    const float* ps[4] = {f.p_l1, f.p_ssim, f.p_sc, f.p_mreg};
    const uint32_t ns[4] = {f.n_l1, f.n_ssim, f.n_sc, f.p_mreg ? f.n_mreg : 0u};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        float acc = 0.0f;
        for (uint32_t i = threadIdx.x; i < ns[k]; i += 256) acc += ps[k][i];
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if ((threadIdx.x & 63) == 0) s_w[k][threadIdx.x >> 6] = acc;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int k = threadIdx.x;
        const float acc = (s_w[k][0] + s_w[k][1]) + (s_w[k][2] + s_w[k][3]);
        f.loss[k] = acc / (float)(k == 2 ? f.P : f.n_img);
    }
}

// FUSED (the native training step): img1 is the clamped image, raw the render before the clamp, and the output is
// the gradient w.r.t. the raw render of (1 - ld) L1 + ld (1 - SSIM): (dSSIM + g_l1 sgn(img1 - img2) / n) where the
// render lies in [0, 1], else 0 -- k_clamp_l1_bwd's expression in the same pass.
// MASK (with FUSED): the L1 term is of clamped * mask, so its gradient reaches the clamped image times the mask, and
// dmask gets l1_scale sgn(clamped * mask - gt) clamped + mreg_scale (mask - 1) (mul's and pow's backward)
template <bool FUSED = false, bool MASK = false>
__global__ void __launch_bounds__(256) k_ssim_bwd_strip(int H, int W, int planes, const float* __restrict__ img1,
                                                        const float* __restrict__ img2, const float* __restrict__ dL,
                                                        float dl_value, const float* __restrict__ dmu1,
                                                        const float* __restrict__ ds1, const float* __restrict__ ds12,
                                                        float* __restrict__ dimg1, const float* __restrict__ raw = nullptr,
                                                        float l1_scale = 0.0f, LossFinal lf = {}, uint32_t lblk = 0,
                                                        const float* __restrict__ mask = nullptr,
                                                        float* __restrict__ dmask = nullptr, float mreg_scale = 0.0f,
                                                        const float* __restrict__ dl_mean = nullptr,
                                                        uint32_t n_mean = 1u) {
    // lblk = 1: block 0 computes the step's loss (dispatched first, beside the strips), the strips follow
    if (lblk && blockIdx.x == 0) { loss_final_block(lf); return; }
    // dl_mean: the gradient of the map's mean (device scalar) -- dL/dmap = *dl_mean / numel, torch's mean backward
    if (dl_mean) dl_value = dl_mean[0] / (float)n_mean;
    const StripPos sp = strip_of(H, W, planes, lblk);
    if (!sp.valid) return;
    const int lane = threadIdx.x & 63;
    const size_t plane = (size_t)sp.plane * H * W;
    const bool colok = sp.x >= 0 && sp.x < W;
    const int ox = sp.x + 5;
    const bool out_col = lane < SSW_OUT && ox < W;
    auto ld3 = [&](int row, float& s0, float& s1, float& s2) {
        if (colok && row >= 0 && row < H) {
            const size_t gi = plane + (size_t)row * W + sp.x;
            const float l = dL ? dL[gi] : dl_value;  // dL == NULL: a uniform dL/dmap (the mean's backward)
            s0 = dmu1[gi] * l; s1 = ds1[gi] * l; s2 = ds12[gi] * l;
        } else {
            s0 = s1 = s2 = 0.0f;
        }
    };
    float ring[11][3];
    float q0[SSIM_PF], q1[SSIM_PF], q2[SSIM_PF];
#pragma unroll
    for (int p = 0; p < SSIM_PF; p++) ld3(sp.y0 - 5 + p, q0[p], q1[p], q2[p]);
    for (int base = 0; base < SSW_IN; base += 11) {
#pragma unroll
        for (int j = 0; j < 11; j++) {
            const int rr = base + j;
            if (rr < SSW_IN) {
                const float s0 = q0[0], s1 = q1[0], s2 = q2[0];
#pragma unroll
                for (int p = 0; p + 1 < SSIM_PF; p++) {
                    q0[p] = q0[p + 1];
                    q1[p] = q1[p + 1];
                    q2[p] = q2[p + 1];
                }
                ld3(sp.y0 - 5 + rr + SSIM_PF, q0[SSIM_PF - 1], q1[SSIM_PF - 1], q2[SSIM_PF - 1]);
                {
                    const float xs[3] = {s0, s1, s2};
                    hconv11_n<3>(xs, ring[j]);
                }
                const int y = sp.y0 + rr - 10;
                if (rr >= 10 && y < H) {
                    float v0 = 0, v1 = 0, v2 = 0;
#pragma unroll
                    for (int k = 0; k < 11; k++) {
                        const int q = (j + 1 + k) % 11;
                        v0 = fmaf(GW[k], ring[q][0], v0);
                        v1 = fmaf(GW[k], ring[q][1], v1);
                        v2 = fmaf(GW[k], ring[q][2], v2);
                    }
                    if (out_col) {
                        const size_t gi = plane + (size_t)y * W + ox;
                        // FUSED: the clamped image is clamp01f(raw) (the forward wrote exactly that): read raw once
                        const float x = FUSED ? raw[gi] : 0.0f;
                        const float i1 = FUSED ? clamp01f(x) : img1[gi], i2 = img2[gi];
                        float d = v0;
                        d += (i1 * 2.0f) * v1;
                        d += i2 * v2;
                        if (FUSED) {
                            const float mk = MASK ? mask[gi] : 1.0f;
                            const float e = MASK ? i1 * mk - i2 : i1 - i2;
                            const float sg = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
                            const float gl = l1_scale * sg;
                            const float gsum = d + (MASK ? gl * mk : gl);
                            d = (x >= 0.f && x <= 1.f) ? gsum : 0.f;
                            if (MASK) dmask[gi] = gl * i1 + mreg_scale * (mk - 1.0f);
                        }
                        dimg1[gi] = d;
                    }
                }
            }
        }
    }
}

static unsigned ssim_strip_blocks(int planes, int H, int W) {
    const long waves = (long)((W + SSW_OUT - 1) / SSW_OUT) * ((H + SSW_ROWS - 1) / SSW_ROWS) * planes;
    return (unsigned)((waves + 3) / 4);
}
uint32_t ssim_waves(int planes, int H, int W) {
    return (uint32_t)(((W + SSW_OUT - 1) / SSW_OUT) * ((H + SSW_ROWS - 1) / SSW_ROWS) * planes);
}

void launch_ssim_fwd(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2, float* map,
                     float* dmu1, float* ds1, float* ds12, hipStream_t s) {
    if ((size_t)B * CH * H * W == 0) return;
    const unsigned blocks = ssim_strip_blocks(B * CH, H, W);
    if (dmu1)
        k_ssim_fwd_strip<true><<<blocks, 256, 0, s>>>(H, W, B * CH, C1, C2, img1, img2, map, dmu1, ds1, ds12);
    else
        k_ssim_fwd_strip<false><<<blocks, 256, 0, s>>>(H, W, B * CH, C1, C2, img1, img2, map, nullptr, nullptr, nullptr);
}
void launch_ssim_bwd(int B, int CH, int H, int W, const float* img1, const float* img2, const float* dL,
                     const float* dmu1, const float* ds1, const float* ds12, float* dimg1, hipStream_t s,
                     float dl_value) {
    if ((size_t)B * CH * H * W == 0) return;
    k_ssim_bwd_strip<false><<<ssim_strip_blocks(B * CH, H, W), 256, 0, s>>>(H, W, B * CH, img1, img2, dL, dl_value, dmu1,
                                                                        ds1, ds12, dimg1);
}
void launch_ssim_mean(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                      float* dmu1, float* ds1, float* ds12, float* part, float* mean, hipStream_t s) {
    const uint32_t nw = ssim_waves(B * CH, H, W);
    const unsigned blocks = ssim_strip_blocks(B * CH, H, W);
    if (nw) {
        if (dmu1)
            k_ssim_fwd_strip<true, false, false, true><<<blocks, 256, 0, s>>>(H, W, B * CH, C1, C2, img1, img2, nullptr,
                                                                             dmu1, ds1, ds12, nullptr, part);
        else
            k_ssim_fwd_strip<false, false, false, true><<<blocks, 256, 0, s>>>(H, W, B * CH, C1, C2, img1, img2, nullptr,
                                                                              nullptr, nullptr, nullptr, nullptr, part);
    }
    // an empty image: 0 / 0 = nan, as torch's mean of an empty map
    k_mean_parts<<<1, 256, 0, s>>>(part, nw, (uint32_t)((size_t)B * CH * H * W), mean);
}
void launch_ssim_mean_bwd(int B, int CH, int H, int W, const float* img1, const float* img2, const float* dl_mean,
                          const float* dmu1, const float* ds1, const float* ds12, float* dimg1, hipStream_t s) {
    if ((size_t)B * CH * H * W == 0) return;
    k_ssim_bwd_strip<false><<<ssim_strip_blocks(B * CH, H, W), 256, 0, s>>>(
        H, W, B * CH, img1, img2, nullptr, 0.0f, dmu1, ds1, ds12, dimg1, nullptr, 0.0f, LossFinal{}, 0u, nullptr, nullptr,
        0.0f, dl_mean, (uint32_t)((size_t)B * CH * H * W));
}
uint32_t ssim_mean_parts(int B, int CH, int H, int W) { return ssim_waves(B * CH, H, W); }
void launch_mean_parts(const float* part, uint32_t n, uint32_t denom, float* out, hipStream_t s) {
    k_mean_parts<<<1, 256, 0, s>>>(part, n, denom, out);
}
void launch_ssim_fwd_fused(int H, int W, float C1, float C2, const float* raw, const float* gt, float* clamped,
                           float* dmu1, float* ds1, float* ds12, float* part, hipStream_t s, const float* mask) {
    if ((size_t)H * W == 0) return;
    if (mask)
        k_ssim_fwd_strip<true, true, true><<<ssim_strip_blocks(3, H, W), 256, 0, s>>>(
            H, W, 3, C1, C2, raw, gt, nullptr, dmu1, ds1, ds12, clamped, part, mask);
    else
        k_ssim_fwd_strip<true, true><<<ssim_strip_blocks(3, H, W), 256, 0, s>>>(H, W, 3, C1, C2, raw, gt, nullptr, dmu1,
                                                                            ds1, ds12, clamped, part);
}
void launch_ssim_bwd_fused(int H, int W, const float* clamped, const float* gt, const float* raw, float dl_value,
                           float l1_scale, const float* dmu1, const float* ds1, const float* ds12, float* d_raw,
                           hipStream_t s, const LossFinal* lf, const float* mask, float* dmask, float mreg_scale) {
    if ((size_t)H * W == 0) return;
    const uint32_t lb = lf ? 1u : 0u;
    if (mask)
        k_ssim_bwd_strip<true, true><<<ssim_strip_blocks(3, H, W) + lb, 256, 0, s>>>(
            H, W, 3, clamped, gt, nullptr, dl_value, dmu1, ds1, ds12, d_raw, raw, l1_scale, lf ? *lf : LossFinal{}, lb,
            mask, dmask, mreg_scale);
    else
        k_ssim_bwd_strip<true><<<ssim_strip_blocks(3, H, W) + lb, 256, 0, s>>>(H, W, 3, clamped, gt, nullptr, dl_value,
                                                                              dmu1, ds1, ds12, d_raw, raw, l1_scale,
                                                                              lf ? *lf : LossFinal{}, lb);
}

// ------------------------------------------------------------------------------------------------
// sparse Adam (adam.cu:10-38): visible Gaussians only, no bias correction.  Grid-stride, one element
// per lane per step; N*M is up to 45*5e6 so 64-bit indices.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_adam(float* __restrict__ param, const float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v,
                                              const bool* __restrict__ visible, float lr, float b1, float b2,
                                              float eps, uint64_t total, uint32_t M) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!visible[i / M]) continue;
        const float gr = grad[i];
        const float em = fmaf(b1, m[i], (1.0f - b1) * gr);
        const float ev = fmaf(b2, v[i], ((1.0f - b2) * gr) * gr);
        const float step = -lr * em / (sqrtf(ev) + eps);
        param[i] += step;
        m[i] = em;
        v[i] = ev;
    }
}

void launch_adam(float* param, const float* grad, float* m, float* v, const bool* visible, float lr, float b1, float b2,
                 float eps, uint32_t N, uint32_t M, hipStream_t s) {
    const uint64_t total = (uint64_t)N * M;
    if (total == 0 || M == 0) return;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    k_adam<<<(unsigned)blocks, 256, 0, s>>>(param, grad, m, v, visible, lr, b1, b2, eps, total, M);
}

// ------------------------------------------------------------------------------------------------
// simple-knn
// ------------------------------------------------------------------------------------------------
constexpr int KNN_BOX = 1024;

// bbox with the reference's {0,0,0} reduction init (simple_knn.cu:191)
__global__ void __launch_bounds__(1024) k_knn_bbox(int P, const float* __restrict__ pts, float* __restrict__ bb) {
    __shared__ float s[6][16];
    float mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    for (int i = threadIdx.x; i < P; i += 1024)
        for (int k = 0; k < 3; k++) {
            const float v = pts[3 * i + k];
            mn[k] = fminf(mn[k], v);
            mx[k] = fmaxf(mx[k], v);
        }
    for (int o = 32; o > 0; o >>= 1)
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], o));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], o));
        }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; k++) { s[k][w] = mn[k]; s[3 + k][w] = mx[k]; }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int k = threadIdx.x;
        float a = s[k][0], b = s[3 + k][0];
        for (int j = 1; j < 16; j++) { a = fminf(a, s[k][j]); b = fmaxf(b, s[3 + k][j]); }
        bb[k] = a;
        bb[3 + k] = b;
    }
}

__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}
__device__ __forceinline__ uint32_t sat_f2u(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}

__global__ void __launch_bounds__(256) k_knn_morton(int P, const float* __restrict__ pts, const float* __restrict__ bb,
                                                    uint32_t* __restrict__ codes) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    uint32_t c[3];
    for (int k = 0; k < 3; k++) c[k] = prep_morton(sat_f2u(((pts[3 * i + k] - bb[k]) / (bb[3 + k] - bb[k])) * 1023.0f));
    codes[i] = c[0] | (c[1] << 1) | (c[2] << 2);
}

__global__ void __launch_bounds__(256) k_knn_boxes(int P, const float* __restrict__ pts, const uint32_t* __restrict__ order,
                                                   float* __restrict__ boxes) {
    __shared__ float s[6][4];
    const int b = blockIdx.x;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = b * KNN_BOX + threadIdx.x; i < P && i < (b + 1) * KNN_BOX; i += 256) {
        const uint32_t g = order[i];
        for (int k = 0; k < 3; k++) {
            const float v = pts[3 * g + k];
            mn[k] = fminf(mn[k], v);
            mx[k] = fmaxf(mx[k], v);
        }
    }
    for (int o = 32; o > 0; o >>= 1)
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], __shfl_xor(mn[k], o));
            mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], o));
        }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; k++) { s[k][w] = mn[k]; s[3 + k][w] = mx[k]; }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float r = s[k][0];
        for (int j = 1; j < 4; j++) r = k < 3 ? fminf(r, s[k][j]) : fmaxf(r, s[k][j]);
        boxes[6 * b + k] = r;
    }
}

__device__ __forceinline__ void upd3(float rx, float ry, float rz, const float* pt, float* best) {
    const float dx = pt[0] - rx, dy = pt[1] - ry, dz = pt[2] - rz;
    float dist = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
#pragma unroll
    for (int j = 0; j < 3; j++)
        if (best[j] > dist) { const float t = best[j]; best[j] = dist; dist = t; }
}

__global__ void __launch_bounds__(256) k_knn_dist(int P, const float* __restrict__ pts, const uint32_t* __restrict__ order,
                                                  const float* __restrict__ boxes, float* __restrict__ out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const uint32_t me = order[idx];
    const float px = pts[3 * me], py = pts[3 * me + 1], pz = pts[3 * me + 2];
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    const int lo = idx - 3 > 0 ? idx - 3 : 0, hi = idx + 3 < P - 1 ? idx + 3 : P - 1;
    for (int i = lo; i <= hi; i++)
        if (i != idx) upd3(px, py, pz, pts + 3 * order[i], best);
    const float reject = best[2];
    best[0] = best[1] = best[2] = FLT_MAX;
    const int nb = (P + KNN_BOX - 1) / KNN_BOX;
    for (int b = 0; b < nb; b++) {
        const float* bx = boxes + 6 * b;
        float d[3] = {0, 0, 0};
        const float p3[3] = {px, py, pz};
#pragma unroll
        for (int k = 0; k < 3; k++)
            if (p3[k] < bx[k] || p3[k] > bx[3 + k]) d[k] = fminf(fabsf(p3[k] - bx[k]), fabsf(p3[k] - bx[3 + k]));
        const float dist = fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
        if (dist > reject || dist > best[2]) continue;
        const int e = (b + 1) * KNN_BOX < P ? (b + 1) * KNN_BOX : P;
        for (int i = b * KNN_BOX; i < e; i++)
            if (i != idx) upd3(px, py, pz, pts + 3 * order[i], best);
    }
    out[me] = (best[0] + best[1] + best[2]) / 3.0f;
}

size_t knn_temp_bytes(int P) {
    const size_t n = (size_t)(P > 0 ? P : 1);
    const size_t nb = (n + KNN_BOX - 1) / KNN_BOX;
    return 256 + 4 * n * 4 + nb * 6 * 4 + radix_sort_temp_bytes((uint32_t)n) + 1024;
}

void launch_knn(int P, const float* pts, float* out, void* temp, hipStream_t s) {
    if (P <= 0) return;
    char* t = (char*)temp;
    float* bb = (float*)t; t += 256;
    uint32_t* k0 = (uint32_t*)t; t += 4 * (size_t)P;
    uint32_t* v0 = (uint32_t*)t; t += 4 * (size_t)P;
    uint32_t* k1 = (uint32_t*)t; t += 4 * (size_t)P;
    uint32_t* v1 = (uint32_t*)t; t += 4 * (size_t)P;
    const int nb = (P + KNN_BOX - 1) / KNN_BOX;
    float* boxes = (float*)t; t += (size_t)nb * 6 * 4;
    t = (char*)(((uintptr_t)t + 255) & ~(uintptr_t)255);
    k_knn_bbox<<<1, 1024, 0, s>>>(P, pts, bb);
    k_knn_morton<<<(P + 255) / 256, 256, 0, s>>>(P, pts, bb, k0);
    const int which = radix_sort_pairs(k0, v0, k1, v1, nullptr, (uint32_t)P, 0, 32, t, s);
    const uint32_t* order = which ? v1 : v0;
    k_knn_boxes<<<nb, 256, 0, s>>>(P, pts, order, boxes);
    k_knn_dist<<<(P + 255) / 256, 256, 0, s>>>(P, pts, order, boxes, out);
}

}  // namespace gs

// mask_head.hip -- the full-resolution head of the appearance embedding (geometry.mask; the reference module
// conerf/model/gaussian_fields/masks.py:8-54: x = upsample(fusion(...)); x = F.interpolate(x, image_size, "bilinear");
// mask = out_conv(x), out_conv = Conv2d(16, 8, 3, pad 1) -> ReLU -> Conv2d(8, 3, 3, pad 1)), forward and backward.
//
// Through torch this head is the embedding's cost at 1080p: a 16-channel 1920 x 1080 tensor (133 MB) written by the
// resize, im2col GEMMs and col2im for the two convolutions, their weight gradients, and the resize's adjoint as
// gathers -- about 3 ms of the 4.5 ms a masked 1080p iteration spends in the embedding (gpurun_out/r6a/mtrace).
// Here the 16-channel image never exists:
//   k_head_fwd    per 6 x 62 output tile: the bilinear samples of the stage-4 output on the tile + 2 halo into LDS,
//                 conv1 + ReLU on the tile + 1 halo into LDS, conv2 -> the [3, H, W] mask;
//   k_head_bwd_h  per tile: h on the tile (stored by the forward, or recomputed from the samples); dL/dh = [h > 0] conv2^T(dmask)
//                 (dmask on the tile + 1 halo) -> dh [8, H, W]; the tile's partial dW2, db2 (fixed-order sums);
//   k_head_bwd_x  per tile: the samples (tile + 1 halo) and dh (tile + 1 halo) -> the tile's partial dW1, db1 and
//                 dL/dsample = conv1^T(dh) on the tile -> dx [16, H, W];
//   k_head_bwd_u  per stage-4 pixel: the resize's adjoint as a gather over the samples that read it, in a fixed order;
//   launch_rowsum the tiles' partials summed per parameter in a fixed order (mask_conv.hip).
// No atomics: bitwise repeatable for a given shape (the ADMM ranks and the sequential baseline rely on it).
// Weights are wave-uniform scalar loads (SGPR operands), the per-position data in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mask_conv.h"

namespace gs {
namespace {

constexpr int HC = 16, HM = 8, HO = 3;        // sample channels, hidden channels, mask channels
constexpr int TH = 8, TW = 64;                 // output tile of the backward kernels
// The forward's tile: its conv1 covers the tile + 1 halo, (6 + 2) x (60 + 2) = 248 position pairs, one per thread
// (an 8 x 64 tile's 10 x 66 = 330 pairs took two passes at 64% use); its samples, 16 x 10 x 64 floats, are 40 KB:
// 4 blocks per CU (62 columns: 42 KB, 3 blocks)
constexpr int FTH = 6, FTW = 60;
constexpr int HT = 256;                        // threads per block
constexpr int NW1 = HM * HC * 9, NW2 = HO * HM * 9;
constexpr int P_W1 = 0, P_B1 = NW1, P_W2 = NW1 + HM, P_B2 = NW1 + HM + NW2;
constexpr int NPART = NW1 + HM + NW2 + HO;     // 1379 partial sums per tile

// bilinear taps of destination index d (torch's upsample_bilinear2d, align_corners = False, no scale factor):
// src = max(0, scale (d + 0.5) - 0.5), i0 = (int) src, i1 = i0 + (i0 < n - 1), l1 = src - i0, l0 = 1 - l1
__device__ __forceinline__ void taps(int d, int n, float scale, int& i0, int& i1, float& l0, float& l1) {
    float src = fmaf(scale, (float)d + 0.5f, -0.5f);
    src = src < 0.0f ? 0.0f : src;
    i0 = (int)src;
    i1 = i0 + (i0 < n - 1 ? 1 : 0);
    l1 = src - (float)i0;
    l0 = 1.0f - l1;
}

// samples of rows [ry0, ry0 + RR) x cols [rx0, rx0 + RC) of the resized image's channels [ch0, ch0 + NCH) into
// xs[NCH][RR][RC] (0 outside it).  An item is one position x 8 channels (32 loads in flight): the forward's 640
// positions x 16 channels are 5 full passes of the block rather than 2.5 passes of 16 channels
template <int RR, int RC, int NCH = HC>
__device__ __forceinline__ void stage_samples(const HeadArgs& a, int ry0, int rx0, float* xs, int ch0 = 0) {
    static_assert(NCH % 8 == 0, "8 channels per item");
    const size_t hw2 = (size_t)a.h2 * a.w2;
    for (int i = threadIdx.x; i < RR * RC * (NCH / 8); i += HT) {
        const int pos = i % (RR * RC), cg = 8 * (i / (RR * RC));
        const int r = pos / RC, c = pos % RC, y = ry0 + r, x = rx0 + c;
        if (y < 0 || y >= a.H || x < 0 || x >= a.W) {
#pragma unroll
            for (int ch = 0; ch < 8; ch++) xs[((cg + ch) * RR + r) * RC + c] = 0.0f;
            continue;
        }
        int iy0, iy1, ix0, ix1;
        float ly0, ly1, lx0, lx1;
        taps(y, a.h2, a.sh, iy0, iy1, ly0, ly1);
        taps(x, a.w2, a.sw, ix0, ix1, lx0, lx1);
        const size_t o00 = (size_t)iy0 * a.w2 + ix0, o01 = (size_t)iy0 * a.w2 + ix1;
        const size_t o10 = (size_t)iy1 * a.w2 + ix0, o11 = (size_t)iy1 * a.w2 + ix1;
        const float* ub = a.U + (size_t)(ch0 + cg) * hw2;
        float v00[8], v01[8], v10[8], v11[8];
#pragma unroll
        for (int ch = 0; ch < 8; ch++) {
            const float* u = ub + ch * hw2;
            v00[ch] = u[o00]; v01[ch] = u[o01]; v10[ch] = u[o10]; v11[ch] = u[o11];
        }
#pragma unroll
        for (int ch = 0; ch < 8; ch++)
            xs[((cg + ch) * RR + r) * RC + c] = ly0 * (lx0 * v00[ch] + lx1 * v01[ch]) + ly1 * (lx0 * v10[ch] + lx1 * v11[ch]);
    }
}

// The weights are wave-uniform: every product reads them as scalar loads (SGPR operands of v_pk_fma_f32).  Staged in
// LDS as broadcast float4 rows they cost one LDS read per 6 FMAs and made the convolution loops LDS-issue-bound: head
// forward 214 -> 169 us, backward 215 + 255 -> 182 + 225 us with the scalar form (gpurun_out/hw1, same box).
// Two positions of a row at once: v_pk_fma_f32 with the weight broadcast to both halves (each half is the same fmaf
// as the scalar form, so the bits do not change).  Left to itself the compiler paired output channels instead, and
// spent a v_mov per weight building the pairs.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(float w, f2 x, f2 acc) { return __builtin_elementwise_fma((f2)(w), x, acc); }

// conv1 + ReLU at the two positions (r, c), (r, c + 1) of a region whose samples xs[HC][XR][XC] start one row and
// column earlier.  Each output sums its 144 products in the same order whichever pair it is computed in, so the
// forward and the backward's recomputation give the same bits.
template <int XR, int XC>
__device__ __forceinline__ void conv1_pair(const float* b1, const float* __restrict__ k1, const float* xs, int r, int c,
                                           float (&h0)[HM], float (&h1)[HM]) {
    f2 h[HM];
#pragma unroll
    for (int co = 0; co < HM; co++) h[co] = (f2)(b1[co]);
#pragma unroll 1
    for (int ci = 0; ci < HC; ci++) {
#pragma unroll
        for (int ky = 0; ky < 3; ky++) {
            const float* row = xs + (ci * XR + r + ky) * XC + c;
            const f2 xa = {row[0], row[1]}, xb = {row[1], row[2]}, xc = {row[2], row[3]};
#pragma unroll
            for (int co = 0; co < HM; co++) {
                const float* wp = k1 + ((co * HC + ci) * 3 + ky) * 3;
                h[co] = fma2(wp[0], xa, h[co]); h[co] = fma2(wp[1], xb, h[co]); h[co] = fma2(wp[2], xc, h[co]);
            }
        }
    }
#pragma unroll
    for (int co = 0; co < HM; co++) {
        h0[co] = h[co].x > 0.0f ? h[co].x : 0.0f;
        h1[co] = h[co].y > 0.0f ? h[co].y : 0.0f;
    }
}

// sliding-window weight-gradient sums over TH rows x TW columns: acc[ky][kx] = sum_(r, c) g[r][c] in[r + ky][c + kx]
// (rows r of the group: grp, grp + G, ...), bacc = sum g
__device__ __forceinline__ void window_sums(const float* in, int in_stride, const float* g, int g_stride, int grp,
                                            int G, float (&acc)[9], float& bacc) {
#pragma unroll
    for (int k = 0; k < 9; k++) acc[k] = 0.0f;
    bacc = 0.0f;
    for (int r = grp; r < TH; r += G) {
        const float* x0r = in + r * in_stride;
        float w00 = x0r[0], w01 = x0r[1];
        float w10 = x0r[in_stride], w11 = x0r[in_stride + 1];
        float w20 = x0r[2 * in_stride], w21 = x0r[2 * in_stride + 1];
        const float* gr = g + r * g_stride;
#pragma unroll 4
        for (int c = 0; c < TW; c++) {
            const float w02 = x0r[c + 2], w12 = x0r[in_stride + c + 2], w22 = x0r[2 * in_stride + c + 2];
            const float gv = gr[c];
            acc[0] = fmaf(gv, w00, acc[0]); acc[1] = fmaf(gv, w01, acc[1]); acc[2] = fmaf(gv, w02, acc[2]);
            acc[3] = fmaf(gv, w10, acc[3]); acc[4] = fmaf(gv, w11, acc[4]); acc[5] = fmaf(gv, w12, acc[5]);
            acc[6] = fmaf(gv, w20, acc[6]); acc[7] = fmaf(gv, w21, acc[7]); acc[8] = fmaf(gv, w22, acc[8]);
            bacc += gv;
            w00 = w01; w01 = w02; w10 = w11; w11 = w12; w20 = w21; w21 = w22;
        }
    }
}

__global__ void __launch_bounds__(HT) __attribute__((amdgpu_waves_per_eu(2))) k_head_fwd(HeadArgs a) {
    constexpr int XR = FTH + 4, XC = FTW + 4, QR = FTH + 2, QC = FTW + 2;
    // The hidden layer overwrites the samples once every thread has its conv1 outputs in registers (at most one position
    // pair per thread); the biases are scalar loads like the weights.  59 -> 40 KB of LDS, 4 blocks per CU instead of 2
    static_assert(QR * (QC / 2) <= HT && HM * QR * QC <= HC * XR * XC, "one pair per thread; h fits the samples' area");
    __shared__ float smem[HC * XR * XC];
    float* xs = smem;                    // samples, tile + 2 halo
    float* hs = xs;                      // then the hidden layer, tile + 1 halo (0 outside the image: conv2's padding)
    const int tx = blockIdx.x % a.tiles_x, ty = blockIdx.x / a.tiles_x;
    const int y0 = ty * FTH, x0 = tx * FTW;
    stage_samples<XR, XC>(a, y0 - 2, x0 - 2, xs);
    __syncthreads();
    {   // position pair (r, c), (r, c + 1)
        const int i = threadIdx.x;
        const bool act = i < QR * (QC / 2);
        const int r = i / (QC / 2), c = 2 * (i % (QC / 2)), y = y0 - 1 + r, x = x0 - 1 + c;
        float h0[HM], h1[HM];
        if (act) conv1_pair<XR, XC>(a.b1, a.k1, xs, r, c, h0, h1);
        const bool in0 = y >= 0 && y < a.H && x >= 0 && x < a.W, in1 = y >= 0 && y < a.H && x + 1 >= 0 && x + 1 < a.W;
        __syncthreads();   // every thread is past the samples
        if (act) {
#pragma unroll
            for (int co = 0; co < HM; co++) {
                hs[(co * QR + r) * QC + c] = in0 ? h0[co] : 0.0f;
                hs[(co * QR + r) * QC + c + 1] = in1 ? h1[co] : 0.0f;
            }
        }
    }
    __syncthreads();
    const size_t HW = (size_t)a.H * a.W;
    if (a.hid) {   // the tile's hidden layer for the backward (which then neither stages the samples nor runs conv1)
        for (int i = threadIdx.x; i < HM * FTH * FTW; i += HT) {
            const int c = i % FTW, r = (i / FTW) % FTH, co = i / (FTW * FTH), y = y0 + r, x = x0 + c;
            if (y < a.H && x < a.W) a.hid[co * HW + (size_t)y * a.W + x] = hs[(co * QR + r + 1) * QC + c + 1];
        }
    }
    for (int i = threadIdx.x; i < FTH * (FTW / 2); i += HT) {
        const int r = i / (FTW / 2), c = 2 * (i % (FTW / 2)), y = y0 + r, x = x0 + c;
        if (y >= a.H || x >= a.W) continue;
        f2 m[HO];
#pragma unroll
        for (int o = 0; o < HO; o++) m[o] = (f2)(a.b2[o]);
#pragma unroll 1
        for (int co = 0; co < HM; co++) {
#pragma unroll
            for (int ky = 0; ky < 3; ky++) {
                const float* row = hs + (co * QR + r + ky) * QC + c;
                const f2 va = {row[0], row[1]}, vb = {row[1], row[2]}, vc = {row[2], row[3]};
#pragma unroll
                for (int o = 0; o < HO; o++) {
                    const float* wp = a.k2 + ((o * HM + co) * 3 + ky) * 3;
                    m[o] = fma2(wp[0], va, m[o]); m[o] = fma2(wp[1], vb, m[o]); m[o] = fma2(wp[2], vc, m[o]);
                }
            }
        }
        const size_t p = (size_t)y * a.W + x;
#pragma unroll
        for (int o = 0; o < HO; o++) {
            a.mask[o * HW + p] = m[o].x;
            if (x + 1 < a.W) a.mask[o * HW + p + 1] = m[o].y;
        }
    }
}

template <bool HID>   // HID: h from the forward's store (a.hid), else recomputed from the samples
__global__ void __launch_bounds__(HT) __attribute__((amdgpu_waves_per_eu(2))) k_head_bwd_h(HeadArgs a) {
    constexpr int XR = TH + 2, XC = TW + 2;
    constexpr int NP = HO * HM, G = HT / NP;    // dW2: 24 pairs x 10 row groups
    // with HID the samples are not staged and the dW2 row-group sums reuse dmask's and h's area once every thread is
    // past them: 67 -> 25 KB of LDS, 6 blocks per CU instead of 2
    constexpr int XS = HID ? 0 : HC * XR * XC;
    static_assert(G * NP * 10 <= HC * XR * XC && G * NP * 10 <= HO * XR * XC + HM * TH * TW,
                  "the row-group sums reuse the samples' region, or dmask's and h's");
    __shared__ float smem[HM + HO * TW + XS + HO * XR * XC + HM * TH * TW];
    float* sb1 = smem;
    float* colsum = sb1 + HM;
    float* xs = colsum + HO * TW;        // samples, tile + 1 halo; then the dW2 row-group sums
    float* ms = xs + XS;                 // dmask, tile + 1 halo (0 outside the image)
    float* hs = ms + HO * XR * XC;       // hidden on the tile (0 outside the image)
    const int tx = blockIdx.x % a.tiles_x, ty = blockIdx.x / a.tiles_x;
    const int y0 = ty * TH, x0 = tx * TW;
    const size_t HW = (size_t)a.H * a.W;
    if (threadIdx.x < HM) sb1[threadIdx.x] = a.b1[threadIdx.x];
    if (!HID) stage_samples<XR, XC>(a, y0 - 1, x0 - 1, xs);
    for (int i = threadIdx.x; i < XR * XC; i += HT) {
        const int r = i / XC, c = i % XC, y = y0 - 1 + r, x = x0 - 1 + c;
        const bool in = y >= 0 && y < a.H && x >= 0 && x < a.W;
#pragma unroll
        for (int o = 0; o < HO; o++) ms[(o * XR + r) * XC + c] = in ? a.dmask[o * HW + (size_t)y * a.W + x] : 0.0f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TH * (TW / 2); i += HT) {     // owned position pairs
        const int r = i / (TW / 2), c = 2 * (i % (TW / 2)), y = y0 + r, x = x0 + c;
        float h0[HM], h1[HM];
        const bool in0 = y < a.H && x < a.W, in1 = y < a.H && x + 1 < a.W;
        if (HID) {
            const size_t q = in0 ? (size_t)y * a.W + x : 0;
#pragma unroll
            for (int co = 0; co < HM; co++) {
                h0[co] = in0 ? a.hid[co * HW + q] : 0.0f;
                h1[co] = in1 ? a.hid[co * HW + q + 1] : 0.0f;
            }
        } else {
            conv1_pair<XR, XC>(sb1, a.k1, xs, r, c, h0, h1);
        }
#pragma unroll
        for (int co = 0; co < HM; co++) {
            if (!in0) h0[co] = 0.0f;
            if (!in1) h1[co] = 0.0f;
            hs[(co * TH + r) * TW + c] = h0[co];
            hs[(co * TH + r) * TW + c + 1] = h1[co];
        }
        if (!in0) continue;
        // dL/dh = [h > 0] conv2^T(dmask): dh[co][q] = sum_(o, ky, kx) w2[o][co][ky][kx] dmask[o][q - (ky, kx) + 1]
        f2 d[HM];
#pragma unroll
        for (int co = 0; co < HM; co++) d[co] = (f2)(0.0f);
#pragma unroll 1
        for (int o = 0; o < HO; o++) {
#pragma unroll
            for (int ky = 0; ky < 3; ky++) {
                const float* row = ms + (o * XR + r + 2 - ky) * XC + c;
                const f2 m21 = {row[2], row[3]}, m10 = {row[1], row[2]}, m0_ = {row[0], row[1]};
#pragma unroll
                for (int co = 0; co < HM; co++) {
                    const float* wq = a.k2 + ((o * HM + co) * 3 + ky) * 3;   // kx = 0, 1, 2 read c + 2, c + 1, c
                    const float4 w = make_float4(wq[0], wq[1], wq[2], 0.0f);
                    d[co] = fma2(w.x, m21, d[co]); d[co] = fma2(w.y, m10, d[co]); d[co] = fma2(w.z, m0_, d[co]);
                }
            }
        }
        const size_t p = (size_t)y * a.W + x;
#pragma unroll
        for (int co = 0; co < HM; co++) {
            a.dh[co * HW + p] = h0[co] > 0.0f ? d[co].x : 0.0f;
            if (in1) a.dh[co * HW + p + 1] = h1[co] > 0.0f ? d[co].y : 0.0f;
        }
    }
    __syncthreads();
    // dW2[o][co][ky][kx] = sum_q h[co][q] dmask[o][q - (ky, kx) + 1]: the window sums of dmask (tile + 1 halo) against
    // h, with the kernel flipped (window offset k' = 2 - k); db2[o] = sum over the tile's pixels of dmask[o], per
    // column over the rows, then over the columns
    const int t = threadIdx.x, pr = t % NP, grp = t / NP;
    float acc[9], bacc;
    if (grp < G) {
        const int o = pr / HM, co = pr % HM;
        window_sums(ms + o * XR * XC, XC, hs + co * TH * TW, TW, grp, G, acc, bacc);
    }
    if (t < HO * TW) {
        const int o = t / TW, c = t % TW;
        float v = 0.0f;
        for (int r = 0; r < TH; r++) v += ms[(o * XR + r + 1) * XC + c + 1];
        colsum[t] = v;
    }
    float* red = HID ? ms : xs;   // every thread is past the samples
    if (HID) __syncthreads();     // ... and past dmask and h
    if (grp < G) {
#pragma unroll
        for (int k = 0; k < 9; k++) red[(grp * NP + pr) * 10 + k] = acc[k];
    }
    __syncthreads();
    float* prow = a.part + (size_t)blockIdx.x * NPART;
    for (int i = t; i < NP * 9; i += HT) {
        const int p = i / 9, k = i % 9, o = p / HM, co = p % HM;
        float v = red[p * 10 + k];
        for (int gg = 1; gg < G; gg++) v += red[(gg * NP + p) * 10 + k];
        prow[P_W2 + (o * HM + co) * 9 + (8 - k)] = v;     // flipped kernel
    }
    if (t < HO) {
        float v = 0.0f;
        for (int c = 0; c < TW; c++) v += colsum[t * TW + c];
        prow[P_B2 + t] = v;
    }
}

// dW1 over one half of the sample channels (xh: channels [half * 8, half * 8 + 8), tile + 1 halo; ds: dh, tile + 1
// halo): dW1[co][ci][ky][kx] = sum over the tile of dh[co][q] sample[ci][q + (ky, kx) - 1], db1[co] = sum dh[co] (with
// the first half).  A thread owns one input x four hidden channels (3 sample + 4 dh LDS reads per 36 FMAs) over two
// 16-column row segments: 16 slots x 16 groups; the four groups of a wave summed by lane exchange ((g0 + g1) +
// (g2 + g3), the same bits in every lane), the waves in order through LDS.
constexpr int W1_Q = 4, W1_NQ = HM / W1_Q, W1_CH = HC / 2, W1_SLOTS = W1_CH * W1_NQ, W1_G = HT / W1_SLOTS;
constexpr int W1_SEG = 16, W1_ITEMS = TH * (TW / W1_SEG), W1_NV = W1_Q * 10, W1_WAVES = HT / 64;
static_assert(W1_G * W1_SLOTS == HT && W1_SLOTS == 16 && W1_ITEMS % W1_G == 0, "four groups of 16 slots per wave");

__device__ __forceinline__ void head_dw1_half(const float* xh, const float* ds, float* red, int half) {
    constexpr int XR = TH + 2, XC = TW + 2;
    const int t = threadIdx.x, slot = t % W1_SLOTS, grp = t / W1_SLOTS;
    const int q = slot % W1_NQ, cl = slot / W1_NQ;
    float acc[W1_Q][9], bacc[W1_Q];
#pragma unroll
    for (int j = 0; j < W1_Q; j++) {
        bacc[j] = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; k++) acc[j][k] = 0.0f;
    }
    const float* xc = xh + cl * XR * XC;
    const float* dc = ds + (q * W1_Q) * XR * XC + XC + 1;    // the tile's dh (inside the halo)
#pragma unroll 1
    for (int it = grp; it < W1_ITEMS; it += W1_G) {
        const int r = it / (TW / W1_SEG), c0 = (it % (TW / W1_SEG)) * W1_SEG;
        const float* x0r = xc + r * XC + c0;
        float w00 = x0r[0], w01 = x0r[1];
        float w10 = x0r[XC], w11 = x0r[XC + 1];
        float w20 = x0r[2 * XC], w21 = x0r[2 * XC + 1];
        const float* dr = dc + r * XC + c0;
#pragma unroll 4
        for (int c = 0; c < W1_SEG; c++) {
            const float w02 = x0r[c + 2], w12 = x0r[XC + c + 2], w22 = x0r[2 * XC + c + 2];
#pragma unroll
            for (int j = 0; j < W1_Q; j++) {
                const float g = dr[j * XR * XC + c];
                acc[j][0] = fmaf(g, w00, acc[j][0]); acc[j][1] = fmaf(g, w01, acc[j][1]);
                acc[j][2] = fmaf(g, w02, acc[j][2]); acc[j][3] = fmaf(g, w10, acc[j][3]);
                acc[j][4] = fmaf(g, w11, acc[j][4]); acc[j][5] = fmaf(g, w12, acc[j][5]);
                acc[j][6] = fmaf(g, w20, acc[j][6]); acc[j][7] = fmaf(g, w21, acc[j][7]);
                acc[j][8] = fmaf(g, w22, acc[j][8]);
                bacc[j] += g;
            }
            w00 = w01; w01 = w02; w10 = w11; w11 = w12; w20 = w21; w21 = w22;
        }
    }
    // the wave's groups are its lanes l, l + 16, l + 32, l + 48: (g0 + g1) + (g2 + g3), commutative adds, so every lane
    // of a slot holds the same bits
    const int lane = t & 63, wave = t >> 6;
    float* wr = red + (wave * W1_SLOTS + slot) * W1_NV;
#pragma unroll
    for (int j = 0; j < W1_Q; j++) {
#pragma unroll
        for (int k = 0; k < 10; k++) {
            float v = k < 9 ? acc[j][k] : bacc[j];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < W1_SLOTS) wr[j * 10 + k] = v;
        }
    }
}

// the waves' sums of one half in order -> the tile's partial row
__device__ __forceinline__ void head_dw1_store(const float* red, float* prow, int half) {
    for (int i = threadIdx.x; i < W1_SLOTS * W1_NV; i += HT) {
        const int sl = i / W1_NV, e = i % W1_NV, j = e / 10, k = e % 10;
        const int pci = half * W1_CH + sl / W1_NQ, pco = (sl % W1_NQ) * W1_Q + j;
        float v = red[i];
#pragma unroll
        for (int w = 1; w < W1_WAVES; w++) v += red[w * W1_SLOTS * W1_NV + i];
        if (k < 9) prow[P_W1 + (pco * HC + pci) * 9 + k] = v;
        else if (pci == 0) prow[P_B1 + pco] = v;
    }
}

// dL/dsample = conv1^T(dh) and dW1, db1 per tile.  LDS: dh (8 channels, tile + 1 halo), half of the samples at a time
// and the waves' dW1 sums, 52 KB: 3 blocks per CU (all 16 sample channels at once were 63 KB, 2 blocks)
__global__ void __launch_bounds__(HT) k_head_bwd_x(HeadArgs a) {
    constexpr int XR = TH + 2, XC = TW + 2;
    __shared__ float smem[HM * XR * XC + W1_CH * XR * XC + W1_WAVES * W1_SLOTS * W1_NV];
    float* ds = smem;                    // dh, tile + 1 halo (0 outside the image)
    float* xh = ds + HM * XR * XC;       // samples of one channel half, tile + 1 halo
    float* red = xh + W1_CH * XR * XC;   // the waves' dW1 sums
    const int tx = blockIdx.x % a.tiles_x, ty = blockIdx.x / a.tiles_x;
    const int y0 = ty * TH, x0 = tx * TW;
    const size_t HW = (size_t)a.H * a.W;
    stage_samples<XR, XC, W1_CH>(a, y0 - 1, x0 - 1, xh, 0);
    for (int i = threadIdx.x; i < XR * XC; i += HT) {
        const int r = i / XC, c = i % XC, y = y0 - 1 + r, x = x0 - 1 + c;
        const bool in = y >= 0 && y < a.H && x >= 0 && x < a.W;
#pragma unroll
        for (int co = 0; co < HM; co++) ds[(co * XR + r) * XC + c] = in ? a.dh[co * HW + (size_t)y * a.W + x] : 0.0f;
    }
    __syncthreads();
    // dL/dsample = conv1^T(dh): dx[ci][p] = sum_(co, ky, kx) w1[co][ci][ky][kx] dh[co][p - (ky, kx) + 1]
    for (int i = threadIdx.x; i < TH * (TW / 2); i += HT) {
        const int r = i / (TW / 2), c = 2 * (i % (TW / 2)), y = y0 + r, x = x0 + c;
        if (y >= a.H || x >= a.W) continue;
        f2 d[HC];
#pragma unroll
        for (int ci = 0; ci < HC; ci++) d[ci] = (f2)(0.0f);
#pragma unroll 1
        for (int co = 0; co < HM; co++) {
#pragma unroll
            for (int ky = 0; ky < 3; ky++) {
                const float* row = ds + (co * XR + r + 2 - ky) * XC + c;
                const f2 g21 = {row[2], row[3]}, g10 = {row[1], row[2]}, g0_ = {row[0], row[1]};
#pragma unroll
                for (int ci = 0; ci < HC; ci++) {
                    const float* wq = a.k1 + ((co * HC + ci) * 3 + ky) * 3;   // kx = 0, 1, 2 read c + 2, c + 1, c
                    const float4 w = make_float4(wq[0], wq[1], wq[2], 0.0f);
                    d[ci] = fma2(w.x, g21, d[ci]); d[ci] = fma2(w.y, g10, d[ci]); d[ci] = fma2(w.z, g0_, d[ci]);
                }
            }
        }
        const size_t p = (size_t)y * a.W + x;
#pragma unroll
        for (int ci = 0; ci < HC; ci++) {
            a.dx[ci * HW + p] = d[ci].x;
            if (x + 1 < a.W) a.dx[ci * HW + p + 1] = d[ci].y;
        }
    }
    float* prow = a.part + (size_t)blockIdx.x * NPART;
    head_dw1_half(xh, ds, red, 0);
    __syncthreads();                     // every thread is past the first half's samples and has stored its sums
    head_dw1_store(red, prow, 0);
    stage_samples<XR, XC, W1_CH>(a, y0 - 1, x0 - 1, xh, W1_CH);
    __syncthreads();                     // the second half staged, the first half's sums read
    head_dw1_half(xh, ds, red, 1);
    __syncthreads();
    head_dw1_store(red, prow, 1);
}

// the samples (along one axis) that read source index u: candidates around u / scale, each tested with taps(); returns
// the count, writing (destination, weight) pairs in ascending destination order (both taps of a clamped edge sample)
__device__ __forceinline__ int rev_taps(int u, int n_src, int n_dst, float scale, int (&dst)[12], float (&wt)[12]) {
    const float inv = (float)n_dst / (float)n_src;
    int lo = (int)floorf(((float)u - 1.0f) * inv) - 2, hi = (int)ceilf(((float)u + 2.0f) * inv) + 2;
    lo = lo < 0 ? 0 : lo;
    hi = hi > n_dst - 1 ? n_dst - 1 : hi;
    int k = 0;
    for (int d = lo; d <= hi && k < 12; d++) {
        int i0, i1;
        float l0, l1;
        taps(d, n_src, scale, i0, i1, l0, l1);
        if (i0 == u && i1 == u) { dst[k] = d; wt[k] = l0 + l1; k++; }
        else if (i0 == u) { dst[k] = d; wt[k] = l0; k++; }
        else if (i1 == u) { dst[k] = d; wt[k] = l1; k++; }
    }
    return k;
}

// the resize's adjoint: du[ci][uy][ux] = sum over samples (y, x) reading (uy, ux) of wy wx dx[ci][y][x]
__global__ void __launch_bounds__(256) k_head_bwd_u(HeadArgs a) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)a.h2 * a.w2) return;
    const int uy = (int)(idx / a.w2), ux = (int)(idx % a.w2);
    int dy[12], dx[12];
    float wy[12], wx[12];
    const int ny = rev_taps(uy, a.h2, a.H, a.sh, dy, wy);
    const int nx = rev_taps(ux, a.w2, a.W, a.sw, dx, wx);
    const size_t HW = (size_t)a.H * a.W, hw2 = (size_t)a.h2 * a.w2;
    float acc[HC];
#pragma unroll
    for (int ci = 0; ci < HC; ci++) acc[ci] = 0.0f;
    for (int i = 0; i < ny; i++) {
        float rs[HC];
#pragma unroll
        for (int ci = 0; ci < HC; ci++) rs[ci] = 0.0f;
        for (int j = 0; j < nx; j++) {
            const size_t o = (size_t)dy[i] * a.W + dx[j];
#pragma unroll
            for (int ci = 0; ci < HC; ci++) rs[ci] = fmaf(wx[j], a.dx[ci * HW + o], rs[ci]);
        }
#pragma unroll
        for (int ci = 0; ci < HC; ci++) acc[ci] = fmaf(wy[i], rs[ci], acc[ci]);
    }
#pragma unroll
    for (int ci = 0; ci < HC; ci++) a.du[ci * hw2 + idx] = acc[ci];
}

}  // namespace

int mask_head_tiles(int H, int W) { return ((W + TW - 1) / TW) * ((H + TH - 1) / TH); }
int mask_head_nparams() { return NPART; }

void launch_mask_head_fwd(HeadArgs a, hipStream_t st) {
    a.tiles_x = (a.W + FTW - 1) / FTW;
    a.tiles_y = (a.H + FTH - 1) / FTH;
    k_head_fwd<<<a.tiles_x * a.tiles_y, HT, 0, st>>>(a);
}

void launch_mask_head_bwd(HeadArgs a, float* grads, hipStream_t st) {
    a.tiles_x = (a.W + TW - 1) / TW;
    a.tiles_y = (a.H + TH - 1) / TH;
    const int nb = a.tiles_x * a.tiles_y;
    if (a.hid) k_head_bwd_h<true><<<nb, HT, 0, st>>>(a);
    else k_head_bwd_h<false><<<nb, HT, 0, st>>>(a);
    k_head_bwd_x<<<nb, HT, 0, st>>>(a);
    const int64_t nu = (int64_t)a.h2 * a.w2;
    k_head_bwd_u<<<(unsigned)((nu + 255) / 256), 256, 0, st>>>(a);
    launch_rowsum(a.part, nb, NPART, a.part + (size_t)nb * NPART, grads, NPART, nullptr, st);
}

}  // namespace gs

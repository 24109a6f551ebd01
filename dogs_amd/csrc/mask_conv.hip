// mask_conv.hip -- the weight gradient of the appearance embedding's 3x3 convolutions (geometry.mask:
// conerf/model/gaussian_fields/masks.py:8-54, trained by gaussian_trainer.py:392-401, 482-484; mipnerf360.yaml and
// urban3d_admm.yaml switch it on).
//
// The embedding's last convolutions run at the render's full size with few channels (16 -> 8 -> 3 at 1920 x 1080; the
// last upsampling stage 8 -> 16 at 544 x 960).  Their weight gradient is a reduction over ~2M pixels into a few
// hundred weights:  dW[co][ci][ky][kx] = sum_{y,x} dY[co][y][x] X[ci][y+ky-1][x+kx-1],  db[co] = sum dY[co].
// MIOpen's deterministic algorithm for it (a Winograd WrW kernel) takes 83 ms per 1080p call, 200 ms per masked training
// iteration (gpurun_out/mp); its fast algorithms use atomics, so runs and ranks round differently.
//
// Here: pass 1, one block per tile of TR x 64 pixels and channel chunk, stages the tile's input with its one-pixel
// halo and the output gradient in LDS; each thread owns one input x four output channels for its group's 16-column
// row segments and slides a 3 x 3 register window along them (3 X + 4 dY LDS reads per 36 FMAs); the groups are
// summed in a fixed order and the block writes its partial [Cout*Cin*9 + Cout] row.  Pass 2 (launch_rowsum) adds the
// partials over the blocks in a fixed order.  Deterministic for a given shape, no atomics.
// The same file holds the convolution's forward and input gradient (k_conv3x3), so the embedding never calls MIOpen.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mask_conv.h"

namespace gs {
namespace {

// q / d for the small q and d of the staging loops (q, d < 2^16): one multiply-high with m = ceil(2^32 / d).  The
// staging loops issue their loads back to back (unrolled, no loop-carried index), which a runtime division or a
// stepped index kept them from: staged one dependent load at a time, the staging took 2-3x the arithmetic.
__host__ inline uint32_t div_magic(uint32_t d) { return (uint32_t)((((uint64_t)1 << 32) + d - 1) / d); }
__device__ __forceinline__ int div_m(int q, uint32_t m) { return (int)__umulhi((uint32_t)q, m); }

// Stage nrows image rows into LDS, one row per wave and step: row q is channel ch = q / rpc (of the nvalid channels
// from ch0; zeros past them), tile row r = q % rpc at image row gy0 + r, columns gx0 .. gx0 + ncols - 1 (ncols <= 128,
// zeros outside the image) -> dst[ch * ch_stride + r * row_stride + c].  Two phases per batch of B rows: every load
// from a clamped (valid) address with the out-of-image lanes zeroed by a select, then the stores -- no branch
// between a load and the next, so the B rows' loads are in flight together.
// gate (may be nullptr, same layout as src): a value is kept only where gate > 0 -- a ReLU's backward folded into the
// staging of its output gradient (gate = the ReLU's output).
// SHUF: src is [4 C][H / 2][W / 2] read as its pixel shuffle (torch.nn.PixelShuffle(2): channel 4 c + 2 (y & 1) +
// (x & 1) at (y / 2, x / 2) is pixel (y, x) of channel c), the upsampling stages' PixelShuffle folded into the staging.
template <int B, bool GATED = false, bool SHUF = false>
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, size_t HW, int H, int W, int ch0, int nvalid,
                                           int gy0, int gx0, int nrows, int rpc, uint32_t m_rpc, int ncols,
                                           float* dst, int ch_stride, int row_stride, int wave, int lane,
                                           const float* __restrict__ gate = nullptr) {
    static_assert(!(GATED && SHUF), "the gate reads src's own layout");
    const int gxa = gx0 + lane, gxb = gx0 + 64 + lane;
    const bool cola = gxa >= 0 && gxa < W, colb = gxb < W;
    const int gxac = gxa < 0 ? 0 : (gxa >= W ? W - 1 : gxa), gxbc = gxb >= W ? W - 1 : gxb;
    const size_t HWq = HW / 4;
    const int Wq = W / 2;
    const size_t offa = SHUF ? (size_t)(gxac & 1) * HWq + (size_t)(gxac >> 1) : (size_t)gxac;
    const size_t offb = SHUF ? (size_t)(gxbc & 1) * HWq + (size_t)(gxbc >> 1) : (size_t)gxbc;
    for (int base = wave; base < nrows; base += 4 * B) {
        float v0[B], v1[B], g0[B], g1[B];
        uint32_t rok = 0;
#pragma unroll
        for (int b = 0; b < B; b++) {   // loads only: the selects wait for phase 2
            const int q = base + 4 * b, ch = div_m(q, m_rpc), r = q - ch * rpc;
            const int gy = gy0 + r;
            rok |= (q < nrows && ch < nvalid && gy >= 0 && gy < H) ? (1u << b) : 0u;
            const int chc = ch < nvalid ? ch : nvalid - 1, gyc = gy < 0 ? 0 : (gy >= H ? H - 1 : gy);
            const size_t ro = SHUF ? (size_t)(4 * (ch0 + chc) + 2 * (gyc & 1)) * HWq + (size_t)(gyc >> 1) * Wq
                                   : (size_t)(ch0 + chc) * HW + (size_t)gyc * W;
            v0[b] = src[ro + offa];
            v1[b] = src[ro + offb];
            g0[b] = GATED ? gate[ro + offa] : 1.0f;   // compile-time: no branch between the loads
            g1[b] = GATED ? gate[ro + offb] : 1.0f;
        }
#pragma unroll
        for (int b = 0; b < B; b++) {
            const int q = base + 4 * b;
            if (q < nrows) {
                const int ch = div_m(q, m_rpc), r = q - ch * rpc;
                float* d = dst + ch * ch_stride + r * row_stride;
                const bool ok = (rok >> b) & 1u;
                if (lane < ncols) d[lane] = ok && cola && g0[b] > 0.0f ? v0[b] : 0.0f;
                if (64 + lane < ncols) d[64 + lane] = ok && colb && g1[b] > 0.0f ? v1[b] : 0.0f;
            }
        }
    }
}

// Stage the weights of input channels c0 .. c0 + nc - 1 for output channels cob .. cob + 2^lg_nco - 1 as
// wl[(ci 9 + k) 2^lg_nco + co] (the adjoint reads w transposed and flipped); output channels past Cout repeat the last
// one (their results are never stored).  Batched as stage_rows.
template <int B, bool ADJ>
__device__ __forceinline__ void stage_weights_kco(const float* __restrict__ w, int Cin, int Cout, int c0, int nc,
                                                  int cob, int lg_nco, float* wl) {
    const int nco = 1 << lg_nco, n = nc * 9 * nco;
    for (int base = threadIdx.x; base < n; base += 256 * B) {
        float v[B];
#pragma unroll
        for (int b = 0; b < B; b++) {
            const int e = base + 256 * b, q = e >> lg_nco, co = e & (nco - 1);
            const int ci = q / 9 < nc ? q / 9 : nc - 1, k = q - (q / 9) * 9;
            const int o = cob + co < Cout ? cob + co : Cout - 1, i = c0 + ci;
            v[b] = ADJ ? w[((size_t)i * Cout + o) * 9 + 8 - k] : w[((size_t)o * Cin + i) * 9 + k];
        }
#pragma unroll
        for (int b = 0; b < B; b++) {
            const int e = base + 256 * b;
            if (e < n) wl[e] = v[b];
        }
    }
}

constexpr int WG_TC = 64;        // tile columns
constexpr int WG_THREADS = 256;
constexpr int WG_LDS_FLOATS = 16384;   // 64 KB
constexpr int WG_CQ = 4;         // output channels per thread
constexpr int WG_SEG = 16;       // columns per work item (4 per tile row)

// Channel chunks: a block handles up to WG_CI input x WG_CO output channels of one tile, so any channel count fits
// LDS; blockIdx.y enumerates the chunks.  A thread owns one input channel x 4 output channels (36 window sums + 4
// bias sums: 3 input and 4 gradient LDS reads per 36 FMAs) for the work items -- 16-column row segments -- of its
// group; the groups' sums are added in group order.  A weight's sum is one chunk block's per tile, whatever the
// chunking, then the tiles' partials are added in a fixed order.
constexpr int WG_CI = 16, WG_CO = 16;

struct WgradShape {
    int Cin, Cout, H, W, TR, tiles_x, tiles_y, npart;
    int CI, CO, nci, nco;       // chunk sizes (CO a multiple of 4) and counts
    int slots, G;               // threads per group (CI x CO / 4), groups
    int xs_stride, dy_stride;   // LDS channel strides (odd: the per-channel reads of a wave spread over the banks)
    uint32_t m_tr2, m_tr;       // div_magic(TR + 2), div_magic(TR)
};

__host__ __device__ inline int odd_up(int v) { return v | 1; }

WgradShape wgrad_shape(int Cin, int Cout, int H, int W) {
    WgradShape s;
    s.Cin = Cin; s.Cout = Cout; s.H = H; s.W = W;
    s.CI = Cin < WG_CI ? Cin : WG_CI;
    const int co4 = (Cout + WG_CQ - 1) / WG_CQ * WG_CQ;
    s.CO = co4 < WG_CO ? co4 : WG_CO;
    s.nci = (Cin + s.CI - 1) / s.CI;
    s.nco = (Cout + s.CO - 1) / s.CO;
    s.slots = s.CI * (s.CO / WG_CQ);
    s.G = WG_THREADS / s.slots;
    int tr = 16;
    for (; tr > 1; tr--) {
        const int xs = odd_up((tr + 2) * (WG_TC + 2)), dy = odd_up(tr * WG_TC);
        if (s.CI * xs + s.CO * dy <= WG_LDS_FLOATS) break;
    }
    s.TR = tr;
    s.xs_stride = odd_up((tr + 2) * (WG_TC + 2));
    s.dy_stride = odd_up(tr * WG_TC);
    s.tiles_x = (W + WG_TC - 1) / WG_TC;
    s.tiles_y = (H + tr - 1) / tr;
    s.npart = Cout * Cin * 9 + Cout;
    s.m_tr2 = div_magic(tr + 2);
    s.m_tr = div_magic(tr);
    return s;
}

template <bool GATED, bool SHUF>
__global__ void __launch_bounds__(WG_THREADS) k_conv3x3_wgrad_part(WgradShape s, const float* __restrict__ x,
                                                                    const float* __restrict__ dy,
                                                                    const float* __restrict__ gate,
                                                                    float* __restrict__ part) {
    extern __shared__ float lds[];
    const int H = s.H, W = s.W, TR = s.TR;
    const int tx = blockIdx.x % s.tiles_x, ty = blockIdx.x / s.tiles_x;
    const int x0 = tx * WG_TC, y0 = ty * TR;
    const int ci0 = (int)(blockIdx.y % s.nci) * s.CI, co0 = (int)(blockIdx.y / s.nci) * s.CO;
    const int Cin = s.Cin - ci0 < s.CI ? s.Cin - ci0 : s.CI;      // this block's channels
    const int Cout = s.Cout - co0 < s.CO ? s.Cout - co0 : s.CO;
    float* xs = lds;                                   // [CI][TR + 2][66], zero outside the image
    float* ds = lds + s.CI * s.xs_stride;              // [CO][TR][64], zero outside the image and past Cout
    const size_t HW = (size_t)H * W;
    const int xrow = WG_TC + 2;
    const int nx = Cin * (TR + 2) * xrow;
    // one staged row per wave and pass, (channel, row) stepped without a division (a runtime integer division per
    // element made the staging, not the sums, the kernel's cost)
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    stage_rows<8, false, SHUF>(x, HW, H, W, ci0, Cin, y0 - 1, x0 - 1, Cin * (TR + 2), TR + 2, s.m_tr2, xrow, xs,
                               s.xs_stride, xrow,
                  wv, ln);
    stage_rows<8, GATED>(dy, HW, H, W, co0, Cout, y0, x0, s.CO * TR, TR, s.m_tr, WG_TC, ds, s.dy_stride, WG_TC, wv,
                         ln, gate);
    __syncthreads();
    const int nq = s.CO / WG_CQ, slots = s.slots, G = s.G;
    const int t = threadIdx.x, grp = t / slots, slot = t % slots;
    const int q = slot % nq, ci = slot / nq;           // output channels 4q .. 4q + 3 of the chunk
    const bool active = grp < G && ci < Cin;
    float acc[WG_CQ][9], bacc[WG_CQ];
#pragma unroll
    for (int j = 0; j < WG_CQ; j++) {
        bacc[j] = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; k++) acc[j][k] = 0.0f;
    }
    if (active) {
        const float* xc = xs + ci * s.xs_stride;
        const float* dc = ds + (q * WG_CQ) * s.dy_stride;
        const int items = TR * (WG_TC / WG_SEG);
        for (int it = grp; it < items; it += G) {
            const int r = it / (WG_TC / WG_SEG), c0 = (it % (WG_TC / WG_SEG)) * WG_SEG;
            const float* x0r = xc + r * xrow + c0;
            float w00 = x0r[0], w01 = x0r[1];
            float w10 = x0r[xrow], w11 = x0r[xrow + 1];
            float w20 = x0r[2 * xrow], w21 = x0r[2 * xrow + 1];
            const float* dr = dc + r * WG_TC + c0;
#pragma unroll 4
            for (int c = 0; c < WG_SEG; c++) {
                const float w02 = x0r[c + 2], w12 = x0r[xrow + c + 2], w22 = x0r[2 * xrow + c + 2];
#pragma unroll
                for (int j = 0; j < WG_CQ; j++) {
                    const float g = dr[j * s.dy_stride + c];
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
    }
    // the groups' sums in group order through LDS (every thread is past the staged tiles)
    __syncthreads();
    constexpr int NV = WG_CQ * 10;
    if (grp < G) {
#pragma unroll
        for (int j = 0; j < WG_CQ; j++) {
#pragma unroll
            for (int k = 0; k < 9; k++) lds[(grp * slots + slot) * NV + j * 10 + k] = acc[j][k];
            lds[(grp * slots + slot) * NV + j * 10 + 9] = bacc[j];
        }
    }
    __syncthreads();
    float* prow = part + (size_t)blockIdx.x * s.npart;
    for (int i = t; i < slots * NV; i += WG_THREADS) {
        const int sl = i / NV, e = i % NV, j = e / 10, k = e % 10;
        const int pci = sl / nq, pco = (sl % nq) * WG_CQ + j;
        if (pci >= Cin || pco >= Cout) continue;
        float v = lds[i];
        for (int gg = 1; gg < G; gg++) v += lds[gg * slots * NV + i];
        if (k < 9) prow[((co0 + pco) * s.Cin + ci0 + pci) * 9 + k] = v;
        else if (ci0 == 0 && pci == 0) prow[s.Cout * s.Cin * 9 + co0 + pco] = v;
    }
}

// ---- the direct 3x3 convolution: forward, and the data gradient as its adjoint ----
//
// y[o][p] = b[o] + sum_i sum_k w(o, i, k) x[i][p + off(k)] with zero padding.  Deterministic, whatever the process
// (MIOpen's choice of algorithm for the same problem depends on its find database and on what ran before in the
// process).  The adjoint reads the forward's weights transposed and flipped, w'(o, i, k) = w[i][o][8 - k], so
// dx = conv(dy, w') with no repacked copy.
// Mapping: a lane owns one column of R rows for 8 output channels (8R accumulators).  A block's 4 waves split as
// WC channel groups x WR row groups x KS input-channel splits over one 64-column tile.  Per round the block stages
// 8 KS input channels with the halo and their weights for the block's 8 WC output channels in LDS; wave (wc, wr, ks)
// sums the round's channels 8 ks .. 8 ks + 7 (3 (R + 2) input reads and 18 broadcast float4 weight reads per 72R
// FMAs) into a round partial that is then added to its total (two-level summation: the fusion's adjoint sums 2304
// products).  With KS > 1 the waves' totals are added in ks order through LDS.  KS splits the long input-channel
// sums of the small low-resolution convolutions (the fusion and its adjoint at 34 x 60 have ~100-300 blocks
// otherwise: one wave per SIMD walking 256 channels, 232 us per adjoint call).
constexpr int CV_TC = 64, CV_CO = 8, CV_CIB = 8, CV_SROW = CV_TC + 2;
constexpr int CV_WFLOATS = CV_CIB * 4 * 9 * CV_CO;   // weights per round: 8 KS x 9 x 8 WC with KS WC <= 4

struct ConvShape {
    int Cin, Cout, H, W;    // as launched: input -> output channels
    int WC, WR, KS, rows;   // waves: channel groups x row groups x input splits; tile rows = WR * R
    int tiles_x, tiles_y, cblocks;
    int lg_nco;             // log2(8 WC)
    uint32_t m_srows;       // div_magic(rows + 2)
    int relu;               // forward: y = max(y, 0) (the stage's ReLU folded into the store)
};

// SH: the forward reads x as its pixel shuffle (stage_rows SHUF); the adjoint writes y as the pixel unshuffle
// ([4 Cin][H / 2][W / 2]), the input gradient of the shuffle folded into the store.
template <int R, bool ADJ, bool GATED = false, bool SH = false>
__global__ void __launch_bounds__(256) k_conv3x3(ConvShape s, const float* __restrict__ x, const float* __restrict__ w,
                                                  const float* __restrict__ b, float* __restrict__ y,
                                                  const float* __restrict__ gate) {
    extern __shared__ float4 lds4[];
    float4* wl = lds4;                                  // [8 KS][9][8 WC / 4] float4
    float* xl = reinterpret_cast<float*>(lds4 + CV_WFLOATS / 4);   // [8 KS][rows + 2][66]
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int ks = wave % s.KS, wr = (wave / s.KS) % s.WR, wc = wave / (s.KS * s.WR);
    const int tx = blockIdx.x % s.tiles_x, ty = blockIdx.x / s.tiles_x;
    const int x0 = tx * CV_TC, y0 = ty * s.rows;
    const int cob = blockIdx.y * s.WC * CV_CO;          // the block's first output channel
    const int H = s.H, W = s.W, Cin = s.Cin, Cout = s.Cout;
    const size_t HW = (size_t)H * W;
    const int srows = s.rows + 2, sch = srows * CV_SROW, nco = s.WC * CV_CO, nco4 = nco / 4;
    float acc[R][CV_CO];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int j = 0; j < CV_CO; j++) acc[r][j] = 0.0f;
    const bool live = cob + wc * CV_CO < Cout;
    const int per_round = CV_CIB * s.KS;
    for (int c0 = 0; c0 < Cin; c0 += per_round) {
        const int nc = Cin - c0 < per_round ? Cin - c0 : per_round;
        if (c0) __syncthreads();
        stage_rows<8, GATED, SH && !ADJ>(x, HW, H, W, c0, nc, y0 - 1, x0 - 1, nc * srows, srows, s.m_srows, CV_SROW,
                                         xl, sch, CV_SROW, wave, lane, gate);
        stage_weights_kco<4, ADJ>(w, Cin, Cout, c0, nc, cob, s.lg_nco, reinterpret_cast<float*>(wl));
        __syncthreads();
        if (!live) continue;
        const int cb = ks * CV_CIB, ce = nc < cb + CV_CIB ? nc : cb + CV_CIB;
        float part[R][CV_CO];
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int j = 0; j < CV_CO; j++) part[r][j] = 0.0f;
#pragma unroll 1
        for (int ci = cb; ci < ce; ci++) {
            const float* l = xl + ci * sch + wr * R * CV_SROW + lane;
            float v[R + 2][3];
#pragma unroll
            for (int rr = 0; rr < R + 2; rr++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++) v[rr][kx] = l[rr * CV_SROW + kx];
            const float4* wk = wl + ci * 9 * nco4 + wc * 2;
#pragma unroll
            for (int k = 0; k < 9; k++) {
                const float4 wa = wk[k * nco4], wb = wk[k * nco4 + 1];
                const float wj[CV_CO] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
                for (int r = 0; r < R; r++)
#pragma unroll
                    for (int j = 0; j < CV_CO; j++) part[r][j] = fmaf(v[r + k / 3][k % 3], wj[j], part[r][j]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int j = 0; j < CV_CO; j++) acc[r][j] += part[r][j];
    }
    if (s.KS > 1) {   // the splits' totals in ks order
        __syncthreads();
        float* red = xl;
        if (live && ks > 0)
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int j = 0; j < CV_CO; j++) red[wave * (R * CV_CO * 64) + (r * CV_CO + j) * 64 + lane] = acc[r][j];
        __syncthreads();
        if (ks > 0 || !live) return;
        for (int q = 1; q < s.KS; q++)
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int j = 0; j < CV_CO; j++) acc[r][j] += red[(wave + q) * (R * CV_CO * 64) + (r * CV_CO + j) * 64 + lane];
    }
    if (!live) return;
    const int gx = x0 + lane;
    if (gx >= W) return;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int gy = y0 + wr * R + r;
        if (gy >= H) break;
#pragma unroll
        for (int j = 0; j < CV_CO; j++) {
            const int o = cob + wc * CV_CO + j;
            if (o < Cout) {
                const float v = acc[r][j] + (b ? b[o] : 0.0f);
                const size_t at = SH && ADJ ? (size_t)(4 * o + 2 * (gy & 1) + (gx & 1)) * (HW / 4) +
                                                  (size_t)(gy >> 1) * (W / 2) + (size_t)(gx >> 1)
                                            : (size_t)o * HW + (size_t)gy * W + gx;
                y[at] = s.relu && !(v > 0.0f) ? 0.0f : v;
            }
        }
    }
}

}  // namespace

bool conv3x3_supported(int Cin, int Cout, int H, int W) {   // output-channel blocks index grid.y (<= 65535)
    return Cin >= 1 && Cout >= 1 && H >= 1 && W >= 1 && Cin <= 65536 && Cout <= 65536 &&
           (int64_t)Cin * Cout <= (1 << 24) && (int64_t)H * W <= ((int64_t)1 << 31);
}

static size_t conv_lds_bytes(const ConvShape& s, int R) {
    const size_t stage = (size_t)CV_CIB * s.KS * (s.rows + 2) * CV_SROW;
    const size_t red = s.KS > 1 ? (size_t)4 * R * CV_CO * 64 : 0;   // one slot per wave (a group's waves are consecutive)
    return (CV_WFLOATS + (stage > red ? stage : red)) * sizeof(float);
}

void launch_conv3x3(int Cin, int Cout, int H, int W, const float* x, const float* w, const float* b, float* y,
                    bool adjoint, bool relu, const float* gate, bool shuffle, hipStream_t st) {
    const int groups = (Cout + CV_CO - 1) / CV_CO, kmax = (Cin + CV_CIB - 1) / CV_CIB;
    // (R, KS) candidates, most work per wave first: the first with >= 256 blocks (one per CU), else the most blocks.
    // (>= 960 blocks, i.e. more splitting for the small low-resolution layers, measured 3% slower over the network's
    // ten calls, >= 64 9% slower: gpurun_out/mf6.)
    const int cand[9][2] = {{4, 1}, {4, 2}, {4, 4}, {2, 1}, {2, 2}, {2, 4}, {1, 1}, {1, 2}, {1, 4}};
    ConvShape best{};
    int bestR = 1;
    int64_t best_blocks = -1;
    for (const auto& c : cand) {
        const int R = c[0], KS = c[1];
        if (KS > 1 && KS > kmax) continue;
        ConvShape s;
        s.Cin = Cin; s.Cout = Cout; s.H = H; s.W = W; s.KS = KS;
        const int wcmax = 4 / KS;
        s.WC = groups >= wcmax ? wcmax : (groups == 3 ? 4 / KS : groups);
        if (s.WC * KS > 4) s.WC = 4 / KS;
        s.WR = 4 / (KS * s.WC);
        s.rows = s.WR * R;
        s.tiles_x = (W + CV_TC - 1) / CV_TC;
        s.tiles_y = (H + s.rows - 1) / s.rows;
        s.cblocks = (groups + s.WC - 1) / s.WC;
        s.lg_nco = s.WC == 4 ? 5 : s.WC == 2 ? 4 : 3;
        s.m_srows = div_magic((uint32_t)(s.rows + 2));
        const int64_t blocks = (int64_t)s.tiles_x * s.tiles_y * s.cblocks;
        if (blocks > best_blocks) { best = s; bestR = R; best_blocks = blocks; }
        if (blocks >= 256) { best = s; bestR = R; break; }
    }
    best.relu = relu && !adjoint;
    const dim3 grid(best.tiles_x * best.tiles_y, best.cblocks);
    const size_t lds = conv_lds_bytes(best, bestR);
    const float* bb = adjoint ? nullptr : b;
    if (adjoint) {
        if (gate && shuffle) {
            if (bestR == 4) k_conv3x3<4, true, true, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, gate);
            else if (bestR == 2) k_conv3x3<2, true, true, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, gate);
            else k_conv3x3<1, true, true, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, gate);
        } else if (gate) {
            if (bestR == 4) k_conv3x3<4, true, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, gate);
            else if (bestR == 2) k_conv3x3<2, true, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, gate);
            else k_conv3x3<1, true, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, gate);
        } else if (shuffle) {
            if (bestR == 4) k_conv3x3<4, true, false, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else if (bestR == 2) k_conv3x3<2, true, false, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else k_conv3x3<1, true, false, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
        } else {
            if (bestR == 4) k_conv3x3<4, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else if (bestR == 2) k_conv3x3<2, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else k_conv3x3<1, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
        }
    } else {
        if (shuffle) {
            if (bestR == 4) k_conv3x3<4, false, false, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else if (bestR == 2) k_conv3x3<2, false, false, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else k_conv3x3<1, false, false, true><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
        } else {
            if (bestR == 4) k_conv3x3<4, false><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else if (bestR == 2) k_conv3x3<2, false><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
            else k_conv3x3<1, false><<<grid, 256, lds, st>>>(best, x, w, bb, y, nullptr);
        }
    }
}

// Column sums of a [nrows][ncols] array of per-block partials in a fixed order: pass 1 sums each column over nseg
// contiguous row segments (a block covers 64 columns x 4 segments: each wave reads whole 256-B row pieces), pass 2
// adds the segments in order.  nseg follows the shape (~16 rows per segment, rowsum_segments), and a few rows are
// summed in one pass: with 32 segments always, the weight gradient's few-row partials of the wide low-resolution
// layers (6 x 154k for the fusion) wrote and re-read 32 segment rows, and the head's tall, narrow 4050 x 1379 partials
// ran 176 blocks walking 126 rows each (50 us).
// (One wave per column striding over the rows read 64 cache lines per load and took 25-37 us.)
constexpr int RS_SEG_MAX = 256;

// segments: ~16 rows each, at most RS_SEG_MAX and at most 4M floats of segment sums (the wide arrays have few rows)
__host__ __device__ inline int rowsum_segments(int nrows, int ncols) {
    if (nrows < 64) return 1;
    int s = (nrows / 16) & ~3;
    const int cap = (int)((((int64_t)1 << 22) / (ncols > 0 ? ncols : 1)) & ~3);
    if (s > RS_SEG_MAX) s = RS_SEG_MAX;
    if (s > cap) s = cap;
    return s < 4 ? 1 : s;
}

__global__ void __launch_bounds__(256) k_rowsum_seg(const float* __restrict__ part, int nrows, int ncols, int nseg,
                                                     float* __restrict__ seg) {
    const int col = blockIdx.x * 64 + (threadIdx.x & 63);
    const int sg = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (col >= ncols) return;
    const int r0 = (int)((int64_t)nrows * sg / nseg), r1 = (int)((int64_t)nrows * (sg + 1) / nseg);
    float v = 0.0f;
#pragma unroll 8
    for (int r = r0; r < r1; r++) v += part[(size_t)r * ncols + col];
    seg[(size_t)sg * ncols + col] = v;
}

// the segments' sums in order (or, with one segment, the rows themselves)
__global__ void __launch_bounds__(256) k_rowsum_final(const float* __restrict__ seg, int nseg, int ncols, int nsplit,
                                                       float* __restrict__ out_a, float* __restrict__ out_b) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= ncols) return;
    float v = 0.0f;
#pragma unroll 8
    for (int sg = 0; sg < nseg; sg++) v += seg[(size_t)sg * ncols + col];
    if (col < nsplit) out_a[col] = v;
    else out_b[col - nsplit] = v;
}

void launch_rowsum(const float* part, int nrows, int ncols, float* seg, float* out_a, int nsplit, float* out_b,
                   hipStream_t st) {
    const int nseg = rowsum_segments(nrows, ncols);
    if (nseg == 1) {   // few rows: one pass over the partials themselves
        k_rowsum_final<<<(ncols + 255) / 256, 256, 0, st>>>(part, nrows, ncols, nsplit, out_a, out_b);
        return;
    }
    k_rowsum_seg<<<dim3((ncols + 63) / 64, nseg / 4), 256, 0, st>>>(part, nrows, ncols, nseg, seg);
    k_rowsum_final<<<(ncols + 255) / 256, 256, 0, st>>>(seg, nseg, ncols, nsplit, out_a, out_b);
}

size_t rowsum_scratch_floats(int nrows, int ncols) {
    const int nseg = rowsum_segments(nrows, ncols);
    return nseg > 1 ? (size_t)nseg * ncols : 0;
}

size_t conv3x3_wgrad_scratch_bytes(int Cin, int Cout, int H, int W) {
    const WgradShape s = wgrad_shape(Cin, Cout, H, W);
    return ((size_t)s.tiles_x * s.tiles_y * s.npart + rowsum_scratch_floats(s.tiles_x * s.tiles_y, s.npart)) *
           sizeof(float);
}

bool conv3x3_wgrad_supported(int Cin, int Cout) {   // the 16 x 16 channel chunks index grid.y (<= 65535)
    return Cin >= 1 && Cout >= 1 && Cin <= 4000 && Cout <= 4000;
}

void launch_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, const float* gate,
                          bool shuffle, float* dw, float* db, float* scratch, hipStream_t st) {
    const WgradShape s = wgrad_shape(Cin, Cout, H, W);
    const int nblk = s.tiles_x * s.tiles_y;
    // the staged tiles, or the groups' sums (at most 256 x 40 floats) when they are larger
    const int stage = s.CI * s.xs_stride + s.CO * s.dy_stride, sums = WG_THREADS * WG_CQ * 10;
    const size_t lds = (size_t)(stage > sums ? stage : sums) * sizeof(float);
    const dim3 grid(nblk, s.nci * s.nco);
    if (gate && shuffle) k_conv3x3_wgrad_part<true, true><<<grid, WG_THREADS, lds, st>>>(s, x, dy, gate, scratch);
    else if (gate) k_conv3x3_wgrad_part<true, false><<<grid, WG_THREADS, lds, st>>>(s, x, dy, gate, scratch);
    else if (shuffle) k_conv3x3_wgrad_part<false, true><<<grid, WG_THREADS, lds, st>>>(s, x, dy, nullptr, scratch);
    else k_conv3x3_wgrad_part<false, false><<<grid, WG_THREADS, lds, st>>>(s, x, dy, nullptr, scratch);
    launch_rowsum(scratch, nblk, s.npart, scratch + (size_t)nblk * s.npart, dw, Cout * Cin * 9, db, st);
}

}  // namespace gs

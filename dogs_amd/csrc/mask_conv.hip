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
    return s;
}

__global__ void __launch_bounds__(WG_THREADS) k_conv3x3_wgrad_part(WgradShape s, const float* __restrict__ x,
                                                                    const float* __restrict__ dy,
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
    for (int i = threadIdx.x; i < nx; i += WG_THREADS) {
        const int c = i % xrow, r = (i / xrow) % (TR + 2), ci = i / (xrow * (TR + 2));
        const int gy = y0 + r - 1, gx = x0 + c - 1;
        float v = 0.0f;
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = x[(size_t)(ci0 + ci) * HW + (size_t)gy * W + gx];
        xs[ci * s.xs_stride + r * xrow + c] = v;
    }
    const int nd = s.CO * TR * WG_TC;
    for (int i = threadIdx.x; i < nd; i += WG_THREADS) {
        const int c = i % WG_TC, r = (i / WG_TC) % TR, co = i / (WG_TC * TR);
        const int gy = y0 + r, gx = x0 + c;
        float v = 0.0f;
        if (co < Cout && gy < H && gx < W) v = dy[(size_t)(co0 + co) * HW + (size_t)gy * W + gx];
        ds[co * s.dy_stride + r * WG_TC + c] = v;
    }
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
// y[o][p] = b[o] + sum_i sum_k w(o, i, k) x[i][p + off(k)] with zero padding, summed in (i, k) order per chunk of 8
// input channels, the chunks' sums then added in order: deterministic,
// whatever the process (MIOpen's choice of algorithm for the same problem depends on its find database and on what
// ran before in the process).  The adjoint reads the forward's weights transposed and flipped,
// w'(o, i, k) = w[i][o][8 - k], so dx = conv(dy, w') with no repacked copy.
// Mapping: a lane owns one column of R rows for 8 output channels (8R accumulators); a block's 4 waves cover WC
// channel groups x WR row groups of one 64-column tile.  Input channels are staged 8 at a time in LDS with the halo; a
// lane reads its 3 x (R + 2) window (conflict-free, lanes are consecutive columns) and the 72 weights of the channel,
// which are wave-uniform (scalar loads), for 72R FMAs.
constexpr int CV_TC = 64, CV_CO = 8, CV_CIB = 8, CV_SROW = CV_TC + 2;

struct ConvShape {
    int Cin, Cout, H, W;    // as launched: input -> output channels
    int WC, WR, rows;       // channel groups x row groups of waves; tile rows = WR * R
    int tiles_x, tiles_y, cblocks;
};

template <int R, bool ADJ>
__global__ void __launch_bounds__(256) k_conv3x3(ConvShape s, const float* __restrict__ x, const float* __restrict__ w,
                                                  const float* __restrict__ b, float* __restrict__ y) {
    extern __shared__ float lds[];   // [CV_CIB][rows + 2][66]
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int wr = wave % s.WR, wc = wave / s.WR;
    const int tx = blockIdx.x % s.tiles_x, ty = blockIdx.x / s.tiles_x;
    const int x0 = tx * CV_TC, y0 = ty * s.rows;
    const int co0 = (blockIdx.y * s.WC + wc) * CV_CO;
    const int H = s.H, W = s.W, Cin = s.Cin, Cout = s.Cout;
    const size_t HW = (size_t)H * W;
    const int srows = s.rows + 2, sch = srows * CV_SROW;
    float acc[R][CV_CO];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int j = 0; j < CV_CO; j++) acc[r][j] = 0.0f;
    const bool live = co0 < Cout;
    for (int c0 = 0; c0 < Cin; c0 += CV_CIB) {
        const int nc = Cin - c0 < CV_CIB ? Cin - c0 : CV_CIB;
        if (c0) __syncthreads();
        for (int row = wave; row < nc * srows; row += 4) {   // one staged row of 66 per wave and pass
            const int ci = row / srows, r = row - ci * srows;
            const int gy = y0 + r - 1;
            float* dst = lds + ci * sch + r * CV_SROW;
            float v0 = 0.0f, v1 = 0.0f;
            if (gy >= 0 && gy < H) {
                const float* src = x + (size_t)(c0 + ci) * HW + (size_t)gy * W;
                const int gx = x0 + lane - 1, gx1 = x0 + CV_TC - 1 + lane;
                if (gx >= 0 && gx < W) v0 = src[gx];
                if (lane < 2 && gx1 < W) v1 = src[gx1];
            }
            dst[lane] = v0;
            if (lane < 2) dst[CV_TC + lane] = v1;
        }
        __syncthreads();
        if (!live) continue;
        float part[R][CV_CO];   // the chunk's sum, then added to the total: two-level summation (the fusion's
                                // adjoint sums 2304 products; one running sum lost ~2x against MIOpen's GEMM)
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int j = 0; j < CV_CO; j++) part[r][j] = 0.0f;
#pragma unroll 1
        for (int ci = 0; ci < nc; ci++) {
            const float* l = lds + ci * sch + wr * R * CV_SROW + lane;
            float v[R + 2][3];
#pragma unroll
            for (int rr = 0; rr < R + 2; rr++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++) v[rr][kx] = l[rr * CV_SROW + kx];
            const int i = c0 + ci;
#pragma unroll
            for (int j = 0; j < CV_CO; j++) {
                const int o = co0 + j < Cout ? co0 + j : Cout - 1;
                float wk[9];
#pragma unroll
                for (int k = 0; k < 9; k++)
                    wk[k] = ADJ ? w[((size_t)i * Cout + o) * 9 + 8 - k] : w[((size_t)o * Cin + i) * 9 + k];
#pragma unroll
                for (int r = 0; r < R; r++)
#pragma unroll
                    for (int k = 0; k < 9; k++) part[r][j] = fmaf(v[r + k / 3][k % 3], wk[k], part[r][j]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int j = 0; j < CV_CO; j++) acc[r][j] += part[r][j];
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
            const int o = co0 + j;
            if (o < Cout) y[(size_t)o * HW + (size_t)gy * W + gx] = acc[r][j] + (b ? b[o] : 0.0f);
        }
    }
}

}  // namespace

bool conv3x3_supported(int Cin, int Cout, int H, int W) {
    return Cin >= 1 && Cout >= 1 && H >= 1 && W >= 1 && (int64_t)Cin * Cout <= (1 << 24) &&
           (int64_t)H * W <= ((int64_t)1 << 31);
}

void launch_conv3x3(int Cin, int Cout, int H, int W, const float* x, const float* w, const float* b, float* y,
                    bool adjoint, hipStream_t st) {
    ConvShape s;
    s.Cin = Cin; s.Cout = Cout; s.H = H; s.W = W;
    const int groups = (Cout + CV_CO - 1) / CV_CO;
    s.WC = groups >= 4 ? 4 : groups == 3 ? 4 : groups;
    s.WR = 4 / s.WC;
    s.tiles_x = (W + CV_TC - 1) / CV_TC;
    s.cblocks = (groups + s.WC - 1) / s.WC;
    int R = 4;   // the most rows per lane that still gives >= 2 blocks per CU
    for (; R > 1; R /= 2) {
        const int64_t blocks = (int64_t)s.tiles_x * ((H + s.WR * R - 1) / (s.WR * R)) * s.cblocks;
        if (blocks >= 512) break;
    }
    s.rows = s.WR * R;
    s.tiles_y = (H + s.rows - 1) / s.rows;
    const dim3 grid(s.tiles_x * s.tiles_y, s.cblocks);
    const size_t lds = (size_t)CV_CIB * (s.rows + 2) * CV_SROW * sizeof(float);
    const float* bb = adjoint ? nullptr : b;
    if (adjoint) {
        if (R == 4) k_conv3x3<4, true><<<grid, 256, lds, st>>>(s, x, w, bb, y);
        else if (R == 2) k_conv3x3<2, true><<<grid, 256, lds, st>>>(s, x, w, bb, y);
        else k_conv3x3<1, true><<<grid, 256, lds, st>>>(s, x, w, bb, y);
    } else {
        if (R == 4) k_conv3x3<4, false><<<grid, 256, lds, st>>>(s, x, w, bb, y);
        else if (R == 2) k_conv3x3<2, false><<<grid, 256, lds, st>>>(s, x, w, bb, y);
        else k_conv3x3<1, false><<<grid, 256, lds, st>>>(s, x, w, bb, y);
    }
}

// Column sums of a [nrows][ncols] array of per-block partials in a fixed order: pass 1 sums each column over
// RS_SEG contiguous row segments (a block covers 64 columns x 4 segments: each wave reads whole 256-B row pieces),
// pass 2 adds the segments in order.  (One wave per column striding over the rows read 64 cache lines per load and
// took 25-37 us; this takes a few.)
constexpr int RS_SEG = 32;

__global__ void __launch_bounds__(256) k_rowsum_seg(const float* __restrict__ part, int nrows, int ncols,
                                                     float* __restrict__ seg) {
    const int col = blockIdx.x * 64 + (threadIdx.x & 63);
    const int sg = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (col >= ncols) return;
    const int r0 = (int)((int64_t)nrows * sg / RS_SEG), r1 = (int)((int64_t)nrows * (sg + 1) / RS_SEG);
    float v = 0.0f;
    for (int r = r0; r < r1; r++) v += part[(size_t)r * ncols + col];
    seg[(size_t)sg * ncols + col] = v;
}

__global__ void __launch_bounds__(256) k_rowsum_final(const float* __restrict__ seg, int ncols, int nsplit,
                                                       float* __restrict__ out_a, float* __restrict__ out_b) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= ncols) return;
    float v = 0.0f;
#pragma unroll 8
    for (int sg = 0; sg < RS_SEG; sg++) v += seg[(size_t)sg * ncols + col];
    if (col < nsplit) out_a[col] = v;
    else out_b[col - nsplit] = v;
}

void launch_rowsum(const float* part, int nrows, int ncols, float* seg, float* out_a, int nsplit, float* out_b,
                   hipStream_t st) {
    k_rowsum_seg<<<dim3((ncols + 63) / 64, RS_SEG / 4), 256, 0, st>>>(part, nrows, ncols, seg);
    k_rowsum_final<<<(ncols + 255) / 256, 256, 0, st>>>(seg, ncols, nsplit, out_a, out_b);
}

size_t rowsum_scratch_floats(int ncols) { return (size_t)RS_SEG * ncols; }

size_t conv3x3_wgrad_scratch_bytes(int Cin, int Cout, int H, int W) {
    const WgradShape s = wgrad_shape(Cin, Cout, H, W);
    return ((size_t)s.tiles_x * s.tiles_y * s.npart + rowsum_scratch_floats(s.npart)) * sizeof(float);
}

bool conv3x3_wgrad_supported(int Cin, int Cout) {
    return Cin >= 1 && Cout >= 1 && Cin <= 4096 && Cout <= 4096;
}

void launch_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, float* dw, float* db,
                          float* scratch, hipStream_t st) {
    const WgradShape s = wgrad_shape(Cin, Cout, H, W);
    const int nblk = s.tiles_x * s.tiles_y;
    // the staged tiles, or the groups' sums (at most 256 x 40 floats) when they are larger
    const int stage = s.CI * s.xs_stride + s.CO * s.dy_stride, sums = WG_THREADS * WG_CQ * 10;
    const size_t lds = (size_t)(stage > sums ? stage : sums) * sizeof(float);
    k_conv3x3_wgrad_part<<<dim3(nblk, s.nci * s.nco), WG_THREADS, lds, st>>>(s, x, dy, scratch);
    launch_rowsum(scratch, nblk, s.npart, scratch + (size_t)nblk * s.npart, dw, Cout * Cin * 9, db, st);
}

}  // namespace gs

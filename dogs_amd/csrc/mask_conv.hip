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
// Here: pass 1, one block per tile of TR x 64 pixels, stages the tile's input with its one-pixel halo and the output
// gradient in LDS; each thread owns one (ci, co) pair for a set of the tile's rows and slides a 3 x 3 register window
// along each row (1 dY + 3 X LDS reads per 9 FMAs); the row groups are summed in a fixed order and the block writes
// its partial [Cout*Cin*9 + Cout] row.  Pass 2, one wave per weight, sums the partials over the blocks lane-strided
// and then across the wave in a fixed tree.  Deterministic for a given shape, no atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mask_conv.h"

namespace gs {
namespace {

constexpr int WG_TC = 64;        // tile columns
constexpr int WG_THREADS = 256;
constexpr int WG_LDS_FLOATS = 16384;   // 64 KB

struct WgradShape {
    int Cin, Cout, H, W, TR, tiles_x, tiles_y, npart;
    int xs_stride, dy_stride;   // LDS channel strides (odd: the per-channel reads of a wave spread over the banks)
};

__host__ __device__ inline int odd_up(int v) { return v | 1; }

WgradShape wgrad_shape(int Cin, int Cout, int H, int W) {
    WgradShape s;
    s.Cin = Cin; s.Cout = Cout; s.H = H; s.W = W;
    int tr = 16;
    for (; tr > 1; tr--) {
        const int xs = odd_up((tr + 2) * (WG_TC + 2)), dy = odd_up(tr * WG_TC);
        if (Cin * xs + Cout * dy <= WG_LDS_FLOATS) break;
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
    const int Cin = s.Cin, Cout = s.Cout, H = s.H, W = s.W, TR = s.TR;
    const int tx = blockIdx.x % s.tiles_x, ty = blockIdx.x / s.tiles_x;
    const int x0 = tx * WG_TC, y0 = ty * TR;
    float* xs = lds;                                   // [Cin][TR + 2][66], zero outside the image
    float* ds = lds + Cin * s.xs_stride;               // [Cout][TR][64], zero outside the image
    const size_t HW = (size_t)H * W;
    const int xrow = WG_TC + 2;
    const int nx = Cin * (TR + 2) * xrow;
    for (int i = threadIdx.x; i < nx; i += WG_THREADS) {
        const int c = i % xrow, r = (i / xrow) % (TR + 2), ci = i / (xrow * (TR + 2));
        const int gy = y0 + r - 1, gx = x0 + c - 1;
        float v = 0.0f;
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) v = x[(size_t)ci * HW + (size_t)gy * W + gx];
        xs[ci * s.xs_stride + r * xrow + c] = v;
    }
    const int nd = Cout * TR * WG_TC;
    for (int i = threadIdx.x; i < nd; i += WG_THREADS) {
        const int c = i % WG_TC, r = (i / WG_TC) % TR, co = i / (WG_TC * TR);
        const int gy = y0 + r, gx = x0 + c;
        float v = 0.0f;
        if (gy < H && gx < W) v = dy[(size_t)co * HW + (size_t)gy * W + gx];
        ds[co * s.dy_stride + r * WG_TC + c] = v;
    }
    __syncthreads();
    const int P = Cin * Cout;
    // threads -> (pair, row group): G row groups of P pairs when P <= 256, else one group and several pairs per thread
    const int G = P >= WG_THREADS ? 1 : WG_THREADS / P;
    const int t = threadIdx.x;
    const int grp = t / (P >= WG_THREADS ? WG_THREADS : P);
    for (int pbase = 0; pbase < P; pbase += (P >= WG_THREADS ? WG_THREADS : P)) {
        const int pair = pbase + (t % (P >= WG_THREADS ? WG_THREADS : P));
        const bool active = grp < G && pair < P && t < G * (P >= WG_THREADS ? WG_THREADS : P);
        float acc[9], bacc = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; k++) acc[k] = 0.0f;
        if (active) {
            const int co = pair % Cout, ci = pair / Cout;
            const float* xc = xs + ci * s.xs_stride;
            const float* dc = ds + co * s.dy_stride;
            for (int r = grp; r < TR; r += G) {
                const float* x0r = xc + r * xrow;
                float w00 = x0r[0], w01 = x0r[1];
                float w10 = x0r[xrow], w11 = x0r[xrow + 1];
                float w20 = x0r[2 * xrow], w21 = x0r[2 * xrow + 1];
                const float* dr = dc + r * WG_TC;
#pragma unroll 4
                for (int c = 0; c < WG_TC; c++) {
                    const float w02 = x0r[c + 2], w12 = x0r[xrow + c + 2], w22 = x0r[2 * xrow + c + 2];
                    const float g = dr[c];
                    acc[0] = fmaf(g, w00, acc[0]); acc[1] = fmaf(g, w01, acc[1]); acc[2] = fmaf(g, w02, acc[2]);
                    acc[3] = fmaf(g, w10, acc[3]); acc[4] = fmaf(g, w11, acc[4]); acc[5] = fmaf(g, w12, acc[5]);
                    acc[6] = fmaf(g, w20, acc[6]); acc[7] = fmaf(g, w21, acc[7]); acc[8] = fmaf(g, w22, acc[8]);
                    bacc += g;
                    w00 = w01; w01 = w02; w10 = w11; w11 = w12; w20 = w21; w21 = w22;
                }
            }
        }
        float* prow = part + (size_t)blockIdx.x * s.npart;
        const int PP = P >= WG_THREADS ? WG_THREADS : P;
        if (G == 1) {   // one row group (P >= 256 pairs, possibly several per thread): the sums are final
            if (active) {
                const int co = pair % Cout, ci = pair / Cout;
#pragma unroll
                for (int k = 0; k < 9; k++) prow[(co * Cin + ci) * 9 + k] = acc[k];
                if (ci == 0) prow[Cout * Cin * 9 + co] = bacc;
            }
            continue;
        }
        // G > 1 row groups (P < 256: this loop runs once): their sums in group order through LDS, where the staged
        // tiles are no longer read
        __syncthreads();
        if (active) {
#pragma unroll
            for (int k = 0; k < 9; k++) lds[(grp * PP + pair) * 10 + k] = acc[k];
            lds[(grp * PP + pair) * 10 + 9] = bacc;
        }
        __syncthreads();
        for (int i = t; i < PP * 10; i += WG_THREADS) {
            const int pl = i / 10, k = i % 10;
            float v = lds[pl * 10 + k];
            for (int gg = 1; gg < G; gg++) v += lds[(gg * PP + pl) * 10 + k];
            const int co = pl % Cout, ci = pl / Cout;
            if (k < 9) prow[(co * Cin + ci) * 9 + k] = v;
            else if (ci == 0) prow[Cout * Cin * 9 + co] = v;
        }
    }
}

}  // namespace

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
    if (Cin < 1 || Cout < 1 || Cin * Cout > 4096) return false;
    const WgradShape s = wgrad_shape(Cin, Cout, 16, 64);
    return Cin * s.xs_stride + Cout * s.dy_stride <= WG_LDS_FLOATS;
}

void launch_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, float* dw, float* db,
                          float* scratch, hipStream_t st) {
    const WgradShape s = wgrad_shape(Cin, Cout, H, W);
    const int nblk = s.tiles_x * s.tiles_y;
    // the staged tiles, or the row groups' sums (at most 256 x 10 floats) when they are larger
    const int stage = Cin * s.xs_stride + Cout * s.dy_stride;
    const size_t lds = (size_t)(stage > WG_THREADS * 10 ? stage : WG_THREADS * 10) * sizeof(float);
    k_conv3x3_wgrad_part<<<nblk, WG_THREADS, lds, st>>>(s, x, dy, scratch);
    launch_rowsum(scratch, nblk, s.npart, scratch + (size_t)nblk * s.npart, dw, Cout * Cin * 9, db, st);
}

}  // namespace gs

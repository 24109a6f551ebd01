// gs_common.h -- device helpers shared by the gfx950 rasterizer kernels.
//
// Arithmetic contract (see DESIGN.md "Bit-exact keys"): the library is compiled with
// -ffp-contract=off and -fhip-fp32-correctly-rounded-divide-sqrt; every fused multiply-add is an
// explicit fmaf() placed exactly where the CPU oracle (oracle/gs_oracle.c) places it, so the
// per-Gaussian preprocess (depth, means2D, conic, radius, precise tile cull) -- everything that
// decides the (tile, depth, index) keys -- is bit-identical to the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sortscan.h"

#define GS_TILE_X 16
#define GS_TILE_Y 16
#define GS_TILE_PIX 256
#define GS_WAVE 64

namespace gs {

// auxiliary.h:21-38
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                       -1.0925484305920792f, 0.5462742152960396f};
__device__ constexpr float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                       0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                       -0.5900435899266435f};

struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };
// glm::mat3 layout: m[col][row]
struct m3 { float m[3][3]; };

__device__ __forceinline__ m3 m3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                                      float a7, float a8) {
    m3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
// glm operator*(mat3, mat3), product order of type_mat3x3.inl with nvcc-style contraction
__device__ __forceinline__ m3 m3_mul(const m3& A, const m3& B) {
    m3 R;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++)
            R.m[j][i] = fmaf(A.m[2][i], B.m[j][2], fmaf(A.m[1][i], B.m[j][1], A.m[0][i] * B.m[j][0]));
    return R;
}
__device__ __forceinline__ m3 m3_T(const m3& A) {
    m3 R;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++) R.m[j][i] = A.m[i][j];
    return R;
}

// auxiliary.h:69-108 (row-vector convention: x' = m0 x + m4 y + m8 z + m12)
__device__ __forceinline__ f3 tp4x3(f3 p, const float* m) {
    return {fmaf(m[8], p.z, fmaf(m[4], p.y, m[0] * p.x)) + m[12],
            fmaf(m[9], p.z, fmaf(m[5], p.y, m[1] * p.x)) + m[13],
            fmaf(m[10], p.z, fmaf(m[6], p.y, m[2] * p.x)) + m[14]};
}
__device__ __forceinline__ f4 tp4x4(f3 p, const float* m) {
    return {fmaf(m[8], p.z, fmaf(m[4], p.y, m[0] * p.x)) + m[12],
            fmaf(m[9], p.z, fmaf(m[5], p.y, m[1] * p.x)) + m[13],
            fmaf(m[10], p.z, fmaf(m[6], p.y, m[2] * p.x)) + m[14],
            fmaf(m[11], p.z, fmaf(m[7], p.y, m[3] * p.x)) + m[15]};
}
__device__ __forceinline__ f3 tv4x3T(f3 p, const float* m) {
    return {fmaf(m[2], p.z, fmaf(m[1], p.y, m[0] * p.x)),
            fmaf(m[6], p.z, fmaf(m[5], p.y, m[4] * p.x)),
            fmaf(m[10], p.z, fmaf(m[9], p.y, m[8] * p.x))};
}
// auxiliary.h:40-43: the reference's double literals make this a double-precision expression
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// v_cvt_i32_f32 saturates and maps NaN to 0 -- the semantics the oracle restates
__device__ __forceinline__ int f2i(float f) { return (int)f; }

// logf of the precise tile cull (rasterizer_impl.cu:151: logf(co.w / (1/255))): correctly rounded, the closest
// stand-in for CUDA's logf (<= 1 ulp).  The same IEEE double operation sequence as gs_crlogf in oracle/gs_oracle.c
// (log a = e ln2 + 2 atanh s, s = (m - 1)/(m + 1), the atanh series to s^19, one rounding to float), so the kernels
// and the oracle agree bit for bit; correctly rounded on every float in [2^-20, 256) with the two listed exceptions
// (exact log within 3e-16 of a float midpoint).  Round 5's float polynomial was 1-3 ulp off on 7.7% of the
// opacities (profiles/r06_logf_census.json).  Evaluated once per binned Gaussian.
__device__ __forceinline__ float gs_crlogf(float a) {
    if (!(a > 0.0f)) return (a == 0.0f) ? -__builtin_inff() : __builtin_nanf("");
    if (a == __builtin_inff()) return __builtin_inff();
    if (a == 0x1.827a74p-7f) return -0x1.1c2b1ep+2f;
    if (a == 0x1.2f1fd6p+3f) return 0x1.1fcbcep+1f;
    uint32_t u = __float_as_uint(a);
    int e = 0;
    if (u < 0x00800000u) { u = __float_as_uint(a * 8388608.0f); e = -23; }
    e += (int)((u >> 23) & 0xff) - 127;
    uint32_t mu = (u & 0x007fffffu) | 0x3f800000u;
    if (mu > 0x3fb504f3u) { mu -= 0x00800000u; e += 1; }   // m in [sqrt(1/2), sqrt(2))
    const double m = (double)__uint_as_float(mu);
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double p = __builtin_fma(s2, 0.10526315789473684, 0.11764705882352941);
    p = __builtin_fma(s2, p, 0.13333333333333333);
    p = __builtin_fma(s2, p, 0.15384615384615385);
    p = __builtin_fma(s2, p, 0.18181818181818182);
    p = __builtin_fma(s2, p, 0.22222222222222222);
    p = __builtin_fma(s2, p, 0.2857142857142857);
    p = __builtin_fma(s2, p, 0.4);
    p = __builtin_fma(s2, p, 0.6666666666666666);
    const double lm = __builtin_fma(s * s2, p, 2.0 * s);
    const double ed = (double)e;
    return (float)__builtin_fma(ed, 0x1.62e42fefa3800p-1, __builtin_fma(ed, 0x1.ef35793c76730p-45, lm));
}

// The same threshold for the render kernels' 8x8-quadrant masks (quad_mask), which only skip work: a quadrant is
// dropped when even its nearest point is past the threshold by QUAD_MARGIN (0.01), and a pixel there fails the
// per-pixel alpha >= 1/255 test anyway.  So any value within the margin gives the same outputs; the hardware log2
// (v_log_f32, ~1 ulp) of o * 255 is within ~1e-6 of the exact one, and costs 3 VALU per splat lane instead of ~30.
__device__ __forceinline__ float quad_log_thr(float opacity) {
    return __builtin_amdgcn_logf(opacity * 255.0f) * 0.693147182f;
}

// getRect (auxiliary.h:45-55) with the int radius overload
__device__ __forceinline__ void get_rect(float px, float py, int r, int gx, int gy, int& x0, int& y0, int& x1,
                                         int& y1) {
    int a;
    a = f2i((px - (float)r) / (float)GS_TILE_X); a = a > 0 ? a : 0; x0 = a < gx ? a : gx;
    a = f2i((py - (float)r) / (float)GS_TILE_Y); a = a > 0 ? a : 0; y0 = a < gy ? a : gy;
    a = f2i((((px + (float)r) + (float)GS_TILE_X) - 1.0f) / (float)GS_TILE_X); a = a > 0 ? a : 0; x1 = a < gx ? a : gx;
    a = f2i((((py + (float)r) + (float)GS_TILE_Y) - 1.0f) / (float)GS_TILE_Y); a = a > 0 ? a : 0; y1 = a < gy ? a : gy;
}

// max_contrib_power_rect_gaussian_float<PATCH,PATCH> (rasterizer_impl.cu:52-100); PATCH = rect size - 1.
// rcx/rcz = 1 / (PATCH^2 * conic.{x,z}) depend on the Gaussian only: callers that test many rects of one
// Gaussian compute them once (mcp_recips) -- the same correctly rounded values, so the same result bits.
template <int PATCH = 15>
__device__ __forceinline__ float2 mcp_recips(f4 co) {
    return make_float2(1.0f / ((float)(PATCH * PATCH) * co.x), 1.0f / ((float)(PATCH * PATCH) * co.z));
}
template <int PATCH = 15>
__device__ __forceinline__ float max_contrib_power_rc(f4 co, float mx, float my, float rminx, float rminy, float rmaxx,
                                                      float rmaxy, float rcx, float rcz) {
    const float x_min_diff = rminx - mx;
    const float x_left = x_min_diff > 0.0f ? 1.0f : 0.0f;
    const float not_in_x = x_left + (mx > rmaxx ? 1.0f : 0.0f);
    const float y_min_diff = rminy - my;
    const float y_above = y_min_diff > 0.0f ? 1.0f : 0.0f;
    const float not_in_y = y_above + (my > rmaxy ? 1.0f : 0.0f);
    float power = 0.0f;
    if ((not_in_y + not_in_x) > 0.0f) {
        const float px = x_left > 0.0f ? rminx : rmaxx;
        const float py = y_above > 0.0f ? rminy : rmaxy;
        const float dx = copysignf((float)PATCH, x_min_diff);
        const float dy = copysignf((float)PATCH, y_min_diff);
        const float diffx = mx - px, diffy = my - py;
        float ax = fmaf(dx * co.y, diffy, (dx * co.x) * diffx) * rcx;
        float ay = fmaf(dy * co.z, diffy, (dy * co.y) * diffx) * rcz;
        ax = (ax != ax) ? 0.0f : fminf(fmaxf(ax, 0.0f), 1.0f);
        ay = (ay != ay) ? 0.0f : fminf(fmaxf(ay, 0.0f), 1.0f);
        const float tx = not_in_y * ax, ty = not_in_x * ay;
        const float qx = fmaf(tx, dx, px), qy = fmaf(ty, dy, py);
        const float ddx = mx - qx, ddy = my - qy;
        power = fmaf(co.y * ddx, ddy, 0.5f * fmaf(co.z * ddy, ddy, (co.x * ddx) * ddx));
    }
    return power;
}
template <int PATCH = 15>
__device__ __forceinline__ float max_contrib_power(f4 co, float mx, float my, float rminx, float rminy, float rmaxx,
                                                   float rmaxy) {
    const float2 rc = mcp_recips<PATCH>(co);
    return max_contrib_power_rc<PATCH>(co, mx, my, rminx, rminy, rmaxx, rmaxy, rc.x, rc.y);
}

// forward.cu:119-153 (quaternion not normalised in-kernel, :128)
__device__ __forceinline__ m3 quat_to_R(float r, float x, float y, float z) {
    return m3_cols(fmaf(-2.f, fmaf(y, y, z * z), 1.f), 2.f * fmaf(x, y, -(r * z)), 2.f * fmaf(x, z, r * y),
                   2.f * fmaf(x, y, r * z), fmaf(-2.f, fmaf(x, x, z * z), 1.f), 2.f * fmaf(y, z, -(r * x)),
                   2.f * fmaf(x, z, -(r * y)), 2.f * fmaf(y, z, r * x), fmaf(-2.f, fmaf(x, x, y * y), 1.f));
}
__device__ __forceinline__ void cov3d_fwd(f3 s, float mod, f4 q, float* cov) {
    m3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * s.x; S.m[1][1] = mod * s.y; S.m[2][2] = mod * s.z;
    m3 R = quat_to_R(q.x, q.y, q.z, q.w);
    m3 M = m3_mul(S, R);
    m3 Mt = m3_T(M);
    m3 Sig = m3_mul(Mt, M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

// computeCov2D (forward.cu:79-114); optionally returns the intermediates the backward needs
struct Cov2DState { m3 T, W, V; f3 t; float xgm, ygm; };
__device__ __forceinline__ f3 cov2d_fwd(f3 mean, float fx, float fy, float tfx, float tfy, const float* cov3D,
                                        const float* vm, Cov2DState* st) {
    f3 t = tp4x3(mean, vm);
    const float limx = 1.3f * tfx, limy = 1.3f * tfy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float tz2 = t.z * t.z;
    m3 J = m3_cols(fx / t.z, 0.0f, -(fx * t.x) / tz2, 0.0f, fy / t.z, -(fy * t.y) / tz2, 0, 0, 0);
    m3 W = m3_cols(vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]);
    m3 T = m3_mul(W, J);
    m3 V = m3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    m3 A = m3_mul(m3_T(T), m3_T(V));
    m3 cov = m3_mul(A, T);
    if (st) {
        st->T = T; st->W = W; st->V = V; st->t = t;
        st->xgm = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
        st->ygm = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    }
    return {cov.m[0][0], cov.m[0][1], cov.m[1][1]};
}

// Copy n4 float4s global -> LDS with LDS-DMA (global_load_lds_dwordx4) by a 256-thread block: each
// wave-instruction lands 1 KiB at a wave-uniform LDS base + lane*16 with no VGPR round trip, so all of the
// block's loads are in flight at once (a register-staged loop waits out one HBM latency per 16 B per lane).
// The caller's next __syncthreads drains them (vmcnt(0) before the barrier).
__device__ __forceinline__ void stage_lds_dma(float4* dst4, const float4* src4, int n4, int t) {
    const int lane = t & 63;
    for (int i0 = t & ~63; i0 < n4; i0 += 256) {
        if (i0 + lane < n4)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src4 + i0 + lane),
                                             (__attribute__((address_space(3))) void*)(dst4 + i0), 16, 0, 0);
    }
}

// Longest-first launch order of the tiles, by one 1024-thread block.  Per-tile work varies by ~10x across
// an image and a 1080p view has only ~1.6 tiles per resident wave slot, so in raster order a render launch
// ends on a tail of long centre tiles; in descending order the short tiles fill in behind the long ones.
// Counting sort on min(len(tile) / 4, 255); the order within a bucket is unspecified (no output depends on
// the launch order).  Each thread evaluates all of its tiles' lengths up front (their loads in flight
// together) and keeps them in registers for the scatter.
template <typename LenFn>
__device__ __forceinline__ void tile_order_sort(int num_tiles, uint32_t* order, LenFn&& len) {
    constexpr int NB = 256, PER = 16;  // up to 1024 * 16 tiles in registers; more loop in chunks
    __shared__ uint32_t s_hist[NB];
    __shared__ uint32_t s_wsum[NB / 64];
    const int t = threadIdx.x;
    if (t < NB) s_hist[t] = 0u;
    __syncthreads();
    const int chunk = (int)blockDim.x * PER;
    uint32_t b0[PER];  // the keys of the first chunk, kept for the scatter (the only chunk up to 16384 tiles)
    for (int c0 = 0; c0 < num_tiles; c0 += chunk) {
        uint32_t b[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int tile = c0 + k * (int)blockDim.x + t;
            const uint32_t l = tile < num_tiles ? len(tile) >> 2 : 0u;
            b[k] = NB - 1 - (l < NB - 1 ? l : NB - 1);
            if (c0 == 0) b0[k] = b[k];
        }
#pragma unroll
        for (int k = 0; k < PER; k++)
            if (c0 + k * (int)blockDim.x + t < num_tiles) atomicAdd(&s_hist[b[k]], 1u);
    }
    __syncthreads();
    uint32_t v = 0, incl = 0;
    if (t < NB) {
        v = s_hist[t];
        incl = v;
        const int lane = t & 63;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[t >> 6] = incl;
    }
    __syncthreads();
    if (t < NB) {
        uint32_t off = 0;
        for (int w = 0; w < (t >> 6); w++) off += s_wsum[w];
        s_hist[t] = off + incl - v;
    }
    __syncthreads();
    for (int c0 = 0; c0 < num_tiles; c0 += chunk) {
        if (c0 > 0 || num_tiles > chunk) {  // more than one chunk: the keys were not kept, recompute them
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const int tile = c0 + k * (int)blockDim.x + t;
                const uint32_t l = tile < num_tiles ? len(tile) >> 2 : 0u;
                b0[k] = NB - 1 - (l < NB - 1 ? l : NB - 1);
            }
        }
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int tile = c0 + k * (int)blockDim.x + t;
            if (tile < num_tiles) order[atomicAdd(&s_hist[b0[k]], 1u)] = (uint32_t)tile;
        }
    }
}

// The same order (same buckets) from two front pieces of two consecutive launches, ORDER_TILES tiles per block, so
// that no single block walks every tile (the one-block sort's contended LDS atomics took ~25 us at 8160 tiles from a
// 256-thread block, on the phase-2 critical path).  ohist[0, ORDER_NB) holds the bucket counts and
// ohist[ORDER_NB, 2 ORDER_NB) the bucket cursors, both zero before the first piece.
//   order_hist_piece:    the block's tiles' buckets into an LDS histogram, flushed with one atomic per nonempty bucket;
//   order_scatter_piece: (a later launch) bucket starts = exclusive scan of the counts, the block's tiles ranked per
//                        bucket in LDS, one global atomic per (block, bucket) reserves the run, then order[] is written.
// Both need blockDim.x == ORDER_TILES == ORDER_NB and `len` returning the same value for a tile in both launches.
// (ORDER_NB, ORDER_TILES, order_blocks: sortscan.h, shared with the host side)
__device__ __forceinline__ uint32_t order_bucket(uint32_t len) {
    const uint32_t l = len >> 2;
    return (uint32_t)ORDER_NB - 1u - (l < (uint32_t)ORDER_NB - 1u ? l : (uint32_t)ORDER_NB - 1u);
}
template <typename LenFn>
__device__ __forceinline__ void order_hist_piece(int num_tiles, int blk, uint32_t* ohist, uint32_t* s_h, LenFn&& len) {
    const int t = threadIdx.x, tile = blk * ORDER_TILES + t;
    s_h[t] = 0u;
    __syncthreads();
    if (tile < num_tiles) atomicAdd(&s_h[order_bucket(len(tile))], 1u);
    __syncthreads();
    if (s_h[t]) atomicAdd(&ohist[t], s_h[t]);
}
template <typename LenFn>
__device__ __forceinline__ void order_scatter_piece(int num_tiles, int blk, uint32_t* ohist, uint32_t* order,
                                                    uint32_t* s_start, uint32_t* s_cnt, uint32_t* s_w, LenFn&& len) {
    const int t = threadIdx.x, lane = t & 63, tile = blk * ORDER_TILES + t;
    const uint32_t b = tile < num_tiles ? order_bucket(len(tile)) : 0u;
    const uint32_t v = ohist[t];
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[t >> 6] = incl;
    s_cnt[t] = 0u;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < (t >> 6); w++) off += s_w[w];
    s_start[t] = off + incl - v;
    const uint32_t r = tile < num_tiles ? atomicAdd(&s_cnt[b], 1u) : 0u;
    __syncthreads();
    if (s_cnt[t]) s_start[t] += atomicAdd(&ohist[ORDER_NB + t], s_cnt[t]);
    __syncthreads();
    if (tile < num_tiles) order[s_start[b] + r] = (uint32_t)tile;
}

constexpr float LOG2E = 1.4426950408889634f;
// Quadrant refinement of the precise tile cull: an 8x8 quadrant whose best point is below the opacity
// threshold holds no pixel with alpha >= 1/255.  The margin (in log units) keeps the skip conservative
// against rounding of both the rect test and the per-pixel exponent.
constexpr float QUAD_MARGIN = 0.01f;
__device__ __forceinline__ uint32_t quad_mask(f4 co, float mx, float my, float thr, int tx0, int ty0) {
    uint32_t m = 0;
    const float2 rc = mcp_recips<7>(co);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const float x0 = (float)(tx0 + (q & 1) * 8), y0 = (float)(ty0 + (q >> 1) * 8);
        const float p = max_contrib_power_rc<7>(co, mx, my, x0, y0, x0 + 7.0f, y0 + 7.0f, rc.x, rc.y);
        m |= (p <= thr + QUAD_MARGIN) ? (1u << q) : 0u;
    }
    return m;
}

// compositing exponent, identical expression in forward and backward (forward.cu:451, backward.cu:596)
__device__ __forceinline__ float splat_power(float cx, float cy, float cz, float dx, float dy) {
    return fmaf(-0.5f, fmaf(cz * dy, dy, (cx * dx) * dx), -((cy * dx) * dy));
}

// Two pixels of one row (same dy) at once: ext_vector_type(2) arithmetic lowers to gfx950's packed
// v_pk_{fma,mul,add}_f32.  On gfx950 a packed op issues in ~5 cycles for both halves whether or not it
// depends on the previous instruction, while a dependent plain fp32 op costs ~5 cycles for one value
// (tools/ubench_valu.hip) -- so the serial per-pixel compositing chain runs packed.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f bc2(float x) { return (v2f){x, x}; }
__device__ __forceinline__ v2f fma2(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }

// Compositing exponent in base 2 for both pixels of a row pair, as Horner form in dx with the row terms
// shared:  p = dx (A dx + B dy) + C dy^2,  A = -a/2 log2 e, B = -b log2 e, C = -c/2 log2 e, which is the
// reference's  -0.5 (a dx^2 + c dy^2) - b dx dy  (forward.cu:451, backward.cu:596) times log2 e.
// Forward and backward evaluate exactly this expression, so the backward replay sees the forward's
// alpha bit for bit; against a per-term evaluation only the last bits of p differ.
struct SplatExp { float A, B, C; };
__device__ __forceinline__ SplatExp splat_exp_coeffs(float ca, float cb, float cc) {
    return {(-0.5f * LOG2E) * ca, -LOG2E * cb, (-0.5f * LOG2E) * cc};
}
__device__ __forceinline__ v2f splat_power2(float A, float B, float C, v2f dx, float dy) {
    const float bdy = B * dy, cdy2 = (C * dy) * dy;
    return fma2(dx, fma2(bc2(A), dx, bc2(bdy)), bc2(cdy2));
}

// Four pixels per lane as {(c0, rA), (c0, rB), (c1, rA), (c1, rB)}: two columns c0, c0 + 8 of two rows
// rA, rA + 8.  Each packed op's halves are independent rows, and lo + hi gives the two row sums.
typedef float v4f __attribute__((ext_vector_type(4)));
// Per-lane rows of a few floats (Gaussian parameters and gradients) are only 4-B aligned; one dwordx2/x3/x4 access per
// row instead of one dword access per float: a wave's dword access touches up to 64 cache lines, and 45 of them per SH
// row made the per-Gaussian passes bound by the address units.
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
// a 3-float row as one dwordx2 + one dword access (rows are only 4-B aligned)
__device__ __forceinline__ f3 ld3(const float* p) {
    const f2u v = *reinterpret_cast<const f2u*>(p);
    return {v.x, v.y, p[2]};
}
__device__ __forceinline__ void st3(float* p, float x, float y, float z) {
    *reinterpret_cast<f2u*>(p) = f2u{x, y};
    p[2] = z;
}

__device__ __forceinline__ v4f bc4(float x) { return (v4f){x, x, x, x}; }
__device__ __forceinline__ v4f fma4(v4f a, v4f b, v4f c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v4f cat4(v2f lo, v2f hi) { return (v4f){lo.x, lo.y, hi.x, hi.y}; }
__device__ __forceinline__ v2f lo2(v4f v) { return (v2f){v.x, v.y}; }
__device__ __forceinline__ v2f hi2(v4f v) { return (v2f){v.z, v.w}; }
// p = dx (A dx + B dy) + C dy^2 for the 4 pixels; identical per-pixel arithmetic to splat_power2
__device__ __forceinline__ v4f splat_power4(float A, float B, float C, float sx, float sy, v4f pxv, v2f pyv) {
    const v2f dy = bc2(sy) - pyv;
    const v2f bdy = bc2(B) * dy, cdy2 = (bc2(C) * dy) * dy;
    const v4f dx = bc4(sx) - pxv;
    return fma4(dx, fma4(bc4(A), dx, cat4(bdy, bdy)), cat4(cdy2, cdy2));
}

}  // namespace gs

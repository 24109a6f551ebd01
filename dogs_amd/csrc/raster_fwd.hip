// raster_fwd.hip -- forward tile rasterizer for gfx950.
//
// Pipeline (DESIGN.md "Forward"):
//   k_preprocess   per Gaussian: EWA projection, SH->RGB, conic, radius, rect and the *precise* per-tile
//                  cull count (rasterizer_impl.cu:57-190 semantics), depth sort key
//   depth sort     stable radix sort of (depth bits, index) over Gaussians           (sortscan.hip)
//   scan           exclusive scan of the precise counts in depth order -> emission offsets
//   k_emit         per Gaussian in depth order: one (tile id, emission index) instance per kept tile
//   tile sort      stable radix sort by tile id only; input order is (depth, index) so the result is the
//                  reference's (tile, depth bits, index) order, bit for bit
//   k_ranges       per-tile [start, end)
//   k_render_fwd   one wave64 per 16x16 tile, 4 pixels per lane; a batch of 64 splats is held one per
//                  lane and broadcast with v_readlane (no LDS, no block barriers); wave-uniform early exit.
#include <hip/hip_runtime.h>
#include "gs_common.h"
#include "raster.h"

namespace gs {

__device__ __forceinline__ int sat_f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 0x7fffffff;
    if (f <= -2147483648.0f) return (int)0x80000000;
    return (int)f;
}

__device__ __forceinline__ void get_rect_s(float px, float py, int r, int gx, int gy, int& x0, int& y0, int& x1,
                                           int& y1) {
    int a;
    a = sat_f2i((px - (float)r) / (float)GS_TILE_X); a = a > 0 ? a : 0; x0 = a < gx ? a : gx;
    a = sat_f2i((py - (float)r) / (float)GS_TILE_Y); a = a > 0 ? a : 0; y0 = a < gy ? a : gy;
    a = sat_f2i((((px + (float)r) + (float)GS_TILE_X) - 1.0f) / (float)GS_TILE_X); a = a > 0 ? a : 0;
    x1 = a < gx ? a : gx;
    a = sat_f2i((((py + (float)r) + (float)GS_TILE_Y) - 1.0f) / (float)GS_TILE_Y); a = a > 0 ? a : 0;
    y1 = a < gy ? a : gy;
}

// computeColorFromSH (forward.cu:24-76); clamped flags are recomputed by the backward instead of stored
__device__ __forceinline__ f3 sh_to_rgb(f3 pos, const float* campos, int deg, const float* d0, const float* sh,
                                        bool* clamped) {
    f3 dir = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
    const float len = sqrtf(fmaf(dir.z, dir.z, fmaf(dir.y, dir.y, dir.x * dir.x)));
    dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
    float r0 = SH_C0 * d0[0], r1 = SH_C0 * d0[1], r2 = SH_C0 * d0[2];
#define ACC(b, k)                                    \
    {                                                \
        const float bb = (b);                        \
        r0 = fmaf(bb, sh[3 * (k) + 0], r0);          \
        r1 = fmaf(bb, sh[3 * (k) + 1], r1);          \
        r2 = fmaf(bb, sh[3 * (k) + 2], r2);          \
    }
    if (deg > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
        ACC(-SH_C1 * y, 0) ACC(SH_C1 * z, 1) ACC(-SH_C1 * x, 2)
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            ACC(SH_C2[0] * xy, 3)
            ACC(SH_C2[1] * yz, 4)
            ACC(SH_C2[2] * (2.0f * zz - xx - yy), 5)
            ACC(SH_C2[3] * xz, 6)
            ACC(SH_C2[4] * (xx - yy), 7)
            if (deg > 2) {
                ACC(SH_C3[0] * y * (3.0f * xx - yy), 8)
                ACC(SH_C3[1] * xy * z, 9)
                ACC(SH_C3[2] * y * (4.0f * zz - xx - yy), 10)
                ACC(SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), 11)
                ACC(SH_C3[4] * x * (4.0f * zz - xx - yy), 12)
                ACC(SH_C3[5] * z * (xx - yy), 13)
                ACC(SH_C3[6] * x * (xx - 3.0f * yy), 14)
            }
        }
    }
#undef ACC
    r0 += 0.5f; r1 += 0.5f; r2 += 0.5f;
    if (clamped) { clamped[0] = r0 < 0; clamped[1] = r1 < 0; clamped[2] = r2 < 0; }
    return {fmaxf(r0, 0.0f), fmaxf(r1, 0.0f), fmaxf(r2, 0.0f)};
}

// Returns the rect area (0 when culled); fills the geometry outputs for kept Gaussians.
__device__ __forceinline__ uint32_t preprocess_one(const PreArgs& a, int idx) {
    a.radii[idx] = 0;
    a.cnt[idx] = 0;
    a.depthkey[idx] = 0xffffffffu;
    const f3 po = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    // in_frustum (auxiliary.h:150-175)
    const f3 pv = tp4x3(po, a.view);
    if (pv.z <= 0.2f) {
        if (a.prefiltered) atomicOr(a.err, 1u);
        return 0;
    }
    const f4 ph = tp4x4(po, a.proj);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ppx = ph.x * pw, ppy = ph.y * pw;
    float cbuf[6];
    const float* cov3D;
    if (a.cov3D_precomp) {
        cov3D = a.cov3D_precomp + 6 * idx;
    } else {
        const f3 s = {a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]};
        const f4 q = {a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]};
        cov3d_fwd(s, a.scale_mod, q, cbuf);
        cov3D = cbuf;
    }
    f3 cov = cov2d_fwd(po, a.focal_x, a.focal_y, a.tanfovx, a.tanfovy, cov3D, a.view, nullptr);
    const float h_var = 0.3f;
    const float det_cov = fmaf(cov.x, cov.z, -(cov.y * cov.y));
    cov.x += h_var; cov.z += h_var;
    const float det_plus = fmaf(cov.x, cov.z, -(cov.y * cov.y));
    float h_scale = 1.0f;
    if (a.antialiasing) h_scale = sqrtf(fmaxf(0.000025f, det_cov / det_plus));
    const float det = det_plus;
    if (det == 0.0f) return 0;
    const float det_inv = 1.f / det;
    const f3 conic = {cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv};
    const float mid = 0.5f * (cov.x + cov.z);
    const float disc = sqrtf(fmaxf(0.1f, fmaf(mid, mid, -det)));
    const float lambda1 = mid + disc, lambda2 = mid - disc;
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const float px = ndc2pix(ppx, a.W), py = ndc2pix(ppy, a.H);
    const int ir = sat_f2i(my_radius);
    int x0, y0, x1, y1;
    get_rect_s(px, py, ir, a.tiles_x, a.tiles_y, x0, y0, x1, y1);
    const uint32_t area = (uint32_t)(x1 - x0) * (uint32_t)(y1 - y0);
    if (area == 0) return 0;
    f3 col;
    if (a.colors) {
        col = {a.colors[3 * idx], a.colors[3 * idx + 1], a.colors[3 * idx + 2]};
    } else {
        col = sh_to_rgb(po, a.campos, a.D, a.dc + 3 * idx, a.sh ? a.sh + (size_t)idx * a.M * 3 : nullptr, nullptr);
    }
    const float4 co = make_float4(conic.x, conic.y, conic.z, a.opacities[idx] * h_scale);
    a.radii[idx] = ir;
    a.xy[idx] = make_float2(px, py);
    a.co[idx] = co;
    a.rgbi[idx] = make_float4(col.x, col.y, col.z, 1.f / pv.z);
    // precise per-tile cull (duplicateWithKeys, rasterizer_impl.cu:149-179)
    const f4 c4 = {co.x, co.y, co.z, co.w};
    const float thr = gs_logf(co.w / (1.0f / 255.0f));
    uint32_t c = 0;
    for (int ty = y0; ty < y1; ty++)
        for (int tx = x0; tx < x1; tx++) {
            const float pw_ = max_contrib_power(c4, px, py, (float)(tx * GS_TILE_X), (float)(ty * GS_TILE_Y),
                                                (float)((tx + 1) * GS_TILE_X - 1), (float)((ty + 1) * GS_TILE_Y - 1));
            c += (pw_ <= thr) ? 1u : 0u;
        }
    a.cnt[idx] = c;
    a.depthkey[idx] = c > 0 ? __float_as_uint(pv.z) : 0xffffffffu;
    return area;
}

__global__ void __launch_bounds__(256) k_preprocess(PreArgs a) {
    __shared__ unsigned long long s_sum[4];
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t area = 0;
    if (idx < a.P) area = preprocess_one(a, idx);
    unsigned long long v = area;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long s = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
        if (s) atomicAdd(a.rect_sum, s);
    }
}

// emission in depth order: instance e = off[p] + j for the j-th kept tile of Gaussian order[p]
__global__ void __launch_bounds__(256) k_emit(int P, const uint32_t* __restrict__ order,
                                              const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                              const float2* __restrict__ xy, const float4* __restrict__ co,
                                              const int* __restrict__ radii, int tiles_x, int tiles_y,
                                              uint32_t* __restrict__ first_e, uint32_t* __restrict__ tilekey,
                                              uint32_t* __restrict__ eg) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const uint32_t g = order[p];
    if (g >= (uint32_t)P) return;
    const uint32_t c = cnt[g];
    if (c == 0) return;
    uint32_t e = off[p];
    first_e[g] = e;
    const float2 m = xy[g];
    const float4 c4v = co[g];
    const f4 c4 = {c4v.x, c4v.y, c4v.z, c4v.w};
    int x0, y0, x1, y1;
    get_rect_s(m.x, m.y, radii[g], tiles_x, tiles_y, x0, y0, x1, y1);
    const float thr = gs_logf(c4.w / (1.0f / 255.0f));
    const uint32_t e_end = e + c;
    for (int ty = y0; ty < y1 && e < e_end; ty++)
        for (int tx = x0; tx < x1; tx++) {
            const float pw_ = max_contrib_power(c4, m.x, m.y, (float)(tx * GS_TILE_X), (float)(ty * GS_TILE_Y),
                                                (float)((tx + 1) * GS_TILE_X - 1), (float)((ty + 1) * GS_TILE_Y - 1));
            if (pw_ <= thr && e < e_end) {
                tilekey[e] = (uint32_t)(ty * tiles_x + tx);
                eg[e] = g;
                e++;
            }
        }
}

// identifyTileRanges over the sorted (all-valid) tile keys
__global__ void __launch_bounds__(256) k_ranges(uint32_t K, const uint32_t* __restrict__ keys,
                                                uint2* __restrict__ ranges, uint32_t num_tiles) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K) return;
    const uint32_t t = keys[i];
    if (t >= num_tiles) return;
    if (i == 0 || keys[i - 1] != t) ranges[t].x = i;
    if (i == K - 1 || keys[i + 1] != t) ranges[t].y = i + 1;
}

__device__ __forceinline__ float bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ uint32_t bcast_u(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

// renderCUDA (forward.cu:349-501) restructured for wave64: one wave per tile, 4 pixels per lane
// (rows ly, ly+4, ly+8, ly+12), the 64-splat batch lives one splat per lane.
__global__ void __launch_bounds__(256) k_render_fwd(RenderArgs a) {
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= a.num_tiles) return;
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int px = tx * GS_TILE_X + (lane & 15);
    const int py0 = ty * GS_TILE_Y + (lane >> 4);
    const float pxf = (float)px;
    float T[4], C0[4], C1[4], C2[4], Dd[4];
    uint32_t last[4];
    bool done[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        T[k] = 1.0f; C0[k] = C1[k] = C2[k] = Dd[k] = 0.0f; last[k] = 0;
        done[k] = !(px < a.W && (py0 + 4 * k) < a.H);
    }
    const uint2 rg = a.ranges[tile];
    const int n = (int)(rg.y - rg.x);
    for (int base = 0; base < n; base += 64) {
        if (__all(done[0] && done[1] && done[2] && done[3])) break;
        const int j = base + lane;
        float gx = 0, gy = 0, ca = 0, cb = 0, cc = 0, op = 0, cr = 0, cg = 0, cbl = 0, ci = 0;
        if (j < n) {
            const uint32_t e = min(a.s_e[rg.x + j], a.K - 1);
            const uint32_t g = min(a.eg[e], a.P - 1);
            const float2 m = a.xy[g];
            const float4 c4 = a.co[g];
            const float4 q = a.rgbi[g];
            gx = m.x; gy = m.y; ca = c4.x; cb = c4.y; cc = c4.z; op = c4.w;
            cr = q.x; cg = q.y; cbl = q.z; ci = q.w;
        }
        const int cntb = (n - base) < 64 ? (n - base) : 64;
        for (int jj = 0; jj < cntb; jj++) {
            const float sx = bcast(gx, jj), sy = bcast(gy, jj);
            const float sa = bcast(ca, jj), sb = bcast(cb, jj), sc = bcast(cc, jj), so = bcast(op, jj);
            const float sr = bcast(cr, jj), sg = bcast(cg, jj), sbl = bcast(cbl, jj), si = bcast(ci, jj);
            const uint32_t contrib = (uint32_t)(base + jj + 1);
            const float dx = sx - pxf;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float dy = sy - (float)(py0 + 4 * k);
                const float power = splat_power(sa, sb, sc, dx, dy);
                const float alpha = fminf(0.99f, so * __expf(power));
                bool ok = !done[k] && !(power > 0.0f) && !(alpha < (1.0f / 255.0f));
                const float test_T = T[k] * (1 - alpha);
                const bool term = ok && (test_T < 0.0001f);
                done[k] = done[k] || term;
                ok = ok && !term;
                if (ok) {
                    C0[k] = fmaf(sr * alpha, T[k], C0[k]);
                    C1[k] = fmaf(sg * alpha, T[k], C1[k]);
                    C2[k] = fmaf(sbl * alpha, T[k], C2[k]);
                    Dd[k] = fmaf(si * alpha, T[k], Dd[k]);
                    T[k] = test_T;
                    last[k] = contrib;
                }
            }
            if (__all(done[0] && done[1] && done[2] && done[3])) break;
        }
    }
    const size_t HW = (size_t)a.W * a.H;
    uint32_t mx = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int py = py0 + 4 * k;
        if (px < a.W && py < a.H) {
            const size_t pid = (size_t)py * a.W + px;
            a.final_T[pid] = T[k];
            a.n_contrib[pid] = last[k];
            const float o0 = fmaf(T[k], a.bg[0], C0[k]);
            const float o1 = fmaf(T[k], a.bg[1], C1[k]);
            const float o2 = fmaf(T[k], a.bg[2], C2[k]);
            a.out_color[pid] = o0; a.out_color[HW + pid] = o1; a.out_color[2 * HW + pid] = o2;
            a.img_color[pid] = o0; a.img_color[HW + pid] = o1; a.img_color[2 * HW + pid] = o2;
            a.out_invd[pid] = Dd[k];
            a.img_invd[pid] = Dd[k];
            mx = last[k] > mx ? last[k] : mx;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(mx, o);
        mx = y > mx ? y : mx;
    }
    if (lane == 0) a.max_contrib[tile] = mx;
}

// checkFrustum (rasterizer_impl.cu:104-116)
__global__ void __launch_bounds__(256) k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view, bool* __restrict__ present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const f3 po = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
    present[i] = tp4x3(po, view).z > 0.2f;
}

// filter_preprocessCUDA (forward.cu:279-344): radii only, no low-pass filter
__global__ void __launch_bounds__(256) k_filter(PreArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    a.radii[idx] = 0;
    const f3 po = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    if (tp4x3(po, a.view).z <= 0.2f) {
        if (a.prefiltered) atomicOr(a.err, 1u);
        return;
    }
    const f4 ph = tp4x4(po, a.proj);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    float cbuf[6];
    const float* cov3D;
    if (a.cov3D_precomp) {
        cov3D = a.cov3D_precomp + 6 * idx;
    } else {
        const f3 s = {a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]};
        const f4 q = {a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]};
        cov3d_fwd(s, a.scale_mod, q, cbuf);
        cov3D = cbuf;
    }
    const f3 cov = cov2d_fwd(po, a.focal_x, a.focal_y, a.tanfovx, a.tanfovy, cov3D, a.view, nullptr);
    const float det = fmaf(cov.x, cov.z, -(cov.y * cov.y));
    if (det == 0.0f) return;
    const float mid = 0.5f * (cov.x + cov.z);
    const float disc = sqrtf(fmaxf(0.1f, fmaf(mid, mid, -det)));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(mid + disc, mid - disc)));
    int x0, y0, x1, y1;
    get_rect_s(ndc2pix(ph.x * pw, a.W), ndc2pix(ph.y * pw, a.H), sat_f2i(my_radius), a.tiles_x, a.tiles_y, x0, y0, x1, y1);
    if ((x1 - x0) * (y1 - y0) == 0) return;
    a.radii[idx] = sat_f2i(my_radius);
}

void launch_preprocess(const PreArgs& a, hipStream_t s) {
    if (a.P > 0) k_preprocess<<<(a.P + 255) / 256, 256, 0, s>>>(a);
}
void launch_emit(int P, const uint32_t* order, const uint32_t* cnt, const uint32_t* off, const float2* xy,
                 const float4* co, const int* radii, int tiles_x, int tiles_y, uint32_t* first_e, uint32_t* tilekey,
                 uint32_t* eg, hipStream_t s) {
    if (P > 0) k_emit<<<(P + 255) / 256, 256, 0, s>>>(P, order, cnt, off, xy, co, radii, tiles_x, tiles_y, first_e,
                                                      tilekey, eg);
}
void launch_ranges(uint32_t K, const uint32_t* keys, uint2* ranges, uint32_t num_tiles, hipStream_t s) {
    if (K > 0) k_ranges<<<(K + 255) / 256, 256, 0, s>>>(K, keys, ranges, num_tiles);
}
void launch_render_fwd(const RenderArgs& a, hipStream_t s) {
    if (a.num_tiles > 0) k_render_fwd<<<(a.num_tiles + 3) / 4, 256, 0, s>>>(a);
}
void launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t s) {
    if (P > 0) k_mark_visible<<<(P + 255) / 256, 256, 0, s>>>(P, means3D, view, present);
}
void launch_filter(const PreArgs& a, hipStream_t s) {
    if (a.P > 0) k_filter<<<(a.P + 255) / 256, 256, 0, s>>>(a);
}

}  // namespace gs

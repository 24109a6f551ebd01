// raster_fwd.hip -- forward tile rasterizer for gfx950.
//
// Pipeline (DESIGN.md "Forward"):
//   k_preprocess   per Gaussian: EWA projection, SH->RGB, conic, radius, rect and the *precise* per-tile
//                  cull count (rasterizer_impl.cu:57-190 semantics), depth key
//   k_depth_hist   instance counts over coarse depth bins;  k_depth_cut: the depth threshold of the phase-1
//                  prefix (instances of Gaussians nearer than it are a prefix of every tile's list)
//   scan           exclusive scan of the precise counts of the prefix Gaussians (index order) -> emission offsets
//   k_emit         per prefix Gaussian: one (tile id, emission index, depth key) instance per kept tile
//   tile binning   atomic counting sort by tile + per-tile sort into (depth bits, index) order (sortscan.hip):
//                  the reference's (tile, depth bits, index) order, bit for bit
//   k_render_fwd   one wave per 16x16 tile, 4 pixels per lane as two row pairs evaluated with packed fp32
//                  (v_pk_*_f32); a 64-splat batch is staged in wave-private LDS and read back with broadcast
//                  ds_read_b128; splats that cannot reach a quadrant pair skip it; wave-uniform early exit.
#include <type_traits>
#include <hip/hip_runtime.h>
#include "gs_common.h"
#include "raster.h"
#include "sortscan.h"
#include "wave_sort.h"

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
__device__ __forceinline__ f3 sh_to_rgb(f3 pos, const float* campos, int deg, f3 d0, const float* sh,
                                        bool* clamped) {
    f3 dir = {pos.x - campos[0], pos.y - campos[1], pos.z - campos[2]};
    const float len = sqrtf(fmaf(dir.z, dir.z, fmaf(dir.y, dir.y, dir.x * dir.x)));
    dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
    float r0 = SH_C0 * d0.x, r1 = SH_C0 * d0.y, r2 = SH_C0 * d0.z;
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


// ---------------------------------------------------------------------------------------------------
// Wave-cooperative (Gaussian, tile) candidate walk.  Every lane owns a Gaussian with tile rect
// [x0,x1) x [y0,y1) (empty when culled).  The wave's candidates are enumerated in (lane, ty, tx) order --
// the reference's duplicateWithKeys order -- 64 per step, so one huge Gaussian no longer makes all 64
// lanes loop over its whole rect.  visit(owner, tile_x, tile_y, kept, valid, chunk_mask) is called once
// per step for every lane; `kept` is the precise per-tile cull (max_contrib_power <= log(255 o)).
struct CandLDS {
    uint32_t pre[64];     // exclusive prefix of rect areas
    int slot[64];         // per step: the lane whose rect starts at this item of the step (-1: none)
    int w[64], area[64];
    float4 co[64];        // conic.xyz, opacity
    float4 geo[64];       // mean2D.xy, log threshold, 1/rect width
    float4 rc[64];        // max_contrib_power reciprocals (mcp_recips), rect x0, y0 (int bits)
};

// `known`: the kept ballots a previous walk of the same candidates recorded -- known.have(step) (wave-uniform) says
// whether step `step` has one, known.mask(step) is it; such steps skip the per-tile power test.
struct NoKnownKept {
    __device__ __forceinline__ bool have(uint32_t) const { return false; }
    __device__ __forceinline__ uint64_t mask(uint32_t) const { return 0ull; }
};
template <typename Visit, typename Known = NoKnownKept>
__device__ __forceinline__ void wave_candidates(CandLDS& L, int lane, int x0, int y0, int x1, int y1, float mx, float my,
                                                float4 co, float thr, Visit&& visit, const Known& known = Known{}) {
    const uint32_t area = (x1 > x0 && y1 > y0) ? (uint32_t)(x1 - x0) * (uint32_t)(y1 - y0) : 0u;
    const uint32_t incl = wave_incl_scan(area);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    L.pre[lane] = incl - area;
    L.w[lane] = x1 - x0; L.area[lane] = (int)area;
    L.co[lane] = co;
    // per-Gaussian constants of the per-tile test, hoisted out of the candidate loop (same values, same bits)
    const float2 rcp = area ? mcp_recips<15>(f4{co.x, co.y, co.z, co.w}) : make_float2(0.f, 0.f);
    L.geo[lane] = make_float4(mx, my, thr, area ? __builtin_amdgcn_rcpf((float)(x1 - x0)) : 0.f);
    L.rc[lane] = make_float4(rcp.x, rcp.y, __int_as_float(x0), __int_as_float(y0));
    __builtin_amdgcn_wave_barrier();
    const uint32_t my_pre = incl - area;
    int carry = 0;  // owner of the item just before the step
    for (uint32_t i0 = 0; i0 < total; i0 += 64) {
        const uint32_t item = i0 + (uint32_t)lane;
        const bool valid = item < total;
        // owner of each item: the rects starting inside this step mark their start slot with their lane, and an
        // item belongs to the last start at or before it (or to the owner carried over from the previous step).
        // Zero-area lanes start nothing.  Two dependent LDS round trips instead of a 6-level binary search.
        L.slot[lane] = -1;
        if (area && my_pre >= i0 && my_pre - i0 < 64u) L.slot[my_pre - i0] = lane;
        __builtin_amdgcn_wave_barrier();
        const int sv = L.slot[lane];
        const uint64_t starts = __ballot(sv >= 0);
        const uint64_t upto = starts & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
        const int pos = upto ? 63 - __clzll((long long)upto) : -1;
        const int from = __shfl(sv, pos < 0 ? 0 : pos);
        int owner = pos >= 0 ? from : carry;
        carry = __builtin_amdgcn_readlane(owner, 63);
        bool kept = false;
        int tx = 0, ty = 0;
        if (!valid) owner = 0;
        const uint32_t step = i0 >> 6;
        const bool have = known.have(step);  // wave-uniform
        if (valid) {
            const int r = (int)(item - L.pre[owner]);
            const int ww = L.w[owner];
            const float4 g = L.geo[owner];
            const float4 rc = L.rc[owner];
            // r / ww from a float reciprocal, corrected to the exact quotient (r < 2^24, error < 1)
            int qy = (int)((float)r * g.w);
            int rx = r - qy * ww;
            if (rx < 0) { qy--; rx += ww; } else if (rx >= ww) { qy++; rx -= ww; }
            tx = __float_as_int(rc.z) + rx;
            ty = __float_as_int(rc.w) + qy;
            if (have) {
                kept = ((known.mask(step) >> lane) & 1ull) != 0ull;
            } else {
                const float4 c = L.co[owner];
                const float p = max_contrib_power_rc<15>(f4{c.x, c.y, c.z, c.w}, g.x, g.y, (float)(tx * GS_TILE_X),
                                                         (float)(ty * GS_TILE_Y), (float)((tx + 1) * GS_TILE_X - 1),
                                                         (float)((ty + 1) * GS_TILE_Y - 1), rc.x, rc.y);
                kept = p <= g.z;
            }
        }
        visit(owner, tx, ty, kept, valid, item);
    }
    __builtin_amdgcn_wave_barrier();
}

// Returns the tile-rect area (0 when culled); fills the geometry outputs of kept Gaussians.  The colour
// (computeColorFromSH) is not evaluated here: only binned Gaussians need it, and k_bin_emit computes it for them.
// The per-Gaussian inputs of the preprocess, loaded before anything is stored (so a thread's several Gaussians have
// all their loads in flight together).  With PreArgs::raw_* they are GaussianSplatModel's activations of the raw
// parameters (optim.hip k_activate_fwd's expressions), stored by pre_compute for the later consumers.
struct PreIn {
    f3 po, s;
    f4 q;
    float opac, prod;
};
__device__ __forceinline__ PreIn pre_load(const PreArgs& a, int idx) {
    PreIn in;
    in.po = {a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]};
    in.s = {0.f, 0.f, 0.f};
    in.q = {0.f, 0.f, 0.f, 0.f};
    in.prod = 0.0f;
    if (a.raw_o) {
        const float ro = a.raw_o[idx];
        const float rs0 = a.raw_s[3 * idx], rs1 = a.raw_s[3 * idx + 1], rs2 = a.raw_s[3 * idx + 2];
        const float4 x = reinterpret_cast<const float4*>(a.raw_q)[idx];
        in.opac = 1.0f / (1.0f + expf(-ro));
        in.s = {expf(rs0), expf(rs1), expf(rs2)};
        in.prod = (in.s.x * in.s.y) * in.s.z;
        const float d = fmaxf(sqrtf((x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w)), 1e-12f);
        in.q = {x.x / d, x.y / d, x.z / d, x.w / d};
    } else {
        if (!a.cov3D_precomp) {
            in.s = {a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]};
            in.q = {a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]};
        }
        in.opac = a.opacities[idx];
    }
    return in;
}

// Returns the tile-rect area (0 when culled); fills the geometry outputs of kept Gaussians.  The colour
// (computeColorFromSH) is not evaluated here: only binned Gaussians need it, and k_bin_emit computes it for them.
__device__ __forceinline__ uint32_t pre_compute(const PreArgs& a, int idx, const PreIn& in) {
    a.radii[idx] = 0;
    a.depthkey[idx] = 0xffffffffu;
    a.cnt[idx] = 0u;
    a.rcnt[idx] = 0u;
    if (a.raw_o) {  // the activated parameters, for the later consumers (opacities / scales / rotations are outputs)
        const_cast<float*>(a.opacities)[idx] = in.opac;
        float* ss = const_cast<float*>(a.scales);
        ss[3 * idx] = in.s.x; ss[3 * idx + 1] = in.s.y; ss[3 * idx + 2] = in.s.z;
        reinterpret_cast<float4*>(const_cast<float*>(a.rotations))[idx] = make_float4(in.q.x, in.q.y, in.q.z, in.q.w);
    }
    const f3 po = in.po;
    const float opac = in.opac;
    // in_frustum (auxiliary.h:150-175)
    const f3 pv = tp4x3(po, a.view);
    if (pv.z <= 0.2f) {
        if (a.prefiltered) atomicOr(a.err, 1u);
        return 0;
    }
    const f4 ph = tp4x4(po, a.proj);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ppx = ph.x * pw, ppy = ph.y * pw;
    // both sources land in registers (a pointer to either would put the local copy on the stack)
    float cbuf[6];
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) cbuf[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        cov3d_fwd(in.s, a.scale_mod, in.q, cbuf);
    }
    const float* cov3D = cbuf;
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
    const float4 co = make_float4(conic.x, conic.y, conic.z, opac * h_scale);
    a.radii[idx] = ir;
    a.sp[2 * idx] = make_float4(px, py, co.x, co.y);
    a.sp[2 * idx + 1] = make_float4(co.z, co.w, __uint_as_float((uint32_t)x0 | ((uint32_t)x1 << 16)),
                                    __uint_as_float((uint32_t)y0 | ((uint32_t)y1 << 16)));
    a.depthkey[idx] = __float_as_uint(pv.z);
    a.cnt[idx] = area;
    return area;
}

#ifndef DG_PRE_PER_THREAD
#define DG_PRE_PER_THREAD 1
#endif
// Gaussians per thread of k_preprocess (their loads issued together); 2 or 4 measured slower (28 -> 32 us per view)
constexpr int PRE_PT = DG_PRE_PER_THREAD;

// One thread per Gaussian.  Neither the precise per-tile cull nor the colour is computed here: only the binned
// Gaussians need them, and the binning walk (k_bin_count / k_bin_emit) computes them for those.
__global__ void __launch_bounds__(256) k_preprocess(PreArgs a) {
    __shared__ unsigned long long s_sum[4];
    __shared__ float s_prod[4];
    __shared__ uint32_t s_err;
    const int t = threadIdx.x;
    const int base = blockIdx.x * 256 * PRE_PT;
    for (int i = blockIdx.x * 256 + t; i < DH_BINS; i += gridDim.x * 256) a.hist[i] = 0u;  // for k_depth_hist
    for (int i = blockIdx.x * 256 + t; i < a.unf_words; i += gridDim.x * 256) a.unf_rows[i] = 0ull;  // phase-1 render
    if (t == 0) s_err = 0u;
    __syncthreads();
    a.err = &s_err;  // a prefiltered violation flags the block (bit 63 of its part)
    PreIn in[PRE_PT];
#pragma unroll
    for (int k = 0; k < PRE_PT; k++) {
        const int idx = base + k * 256 + t;
        if (idx < a.P) in[k] = pre_load(a, idx);
    }
    uint32_t area = 0;
    float prod = 0.0f;
#pragma unroll
    for (int k = 0; k < PRE_PT; k++) {
        const int idx = base + k * 256 + t;
        if (idx < a.P) {
            area += pre_compute(a, idx, in[k]);
            prod += in[k].prod;
            if (a.zero_stamp && (in[k].s.x == 0.0f || in[k].s.y == 0.0f || in[k].s.z == 0.0f))
                *a.zero_stamp = a.stamp;  // the same value from every writer
        }
    }
    unsigned long long v = area;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        v += __shfl_xor(v, o);
        if (a.part_sc) prod += __shfl_xor(prod, o);
    }
    if ((threadIdx.x & 63) == 0) { s_sum[threadIdx.x >> 6] = v; s_prod[threadIdx.x >> 6] = prod; }
    __syncthreads();
    if (threadIdx.x == 0) {
        a.rect_part[blockIdx.x] = (s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3]) | (s_err ? (1ull << 63) : 0ull);
        if (a.part_sc) a.part_sc[blockIdx.x] = (s_prod[0] + s_prod[1]) + (s_prod[2] + s_prod[3]);
    }
}

// ---------------------------------------------------------------------------------------------------
// Depth-threshold prefix (DESIGN.md "Binning").  Phase 1 bins the Gaussians whose depth key is below a
// threshold `thr`; because every tile's list is in (depth bits, index) order, those instances are a PREFIX of
// every tile's list, whatever the threshold.  thr is picked from a histogram of tile-rect areas (an upper bound
// of the precise instance counts) over coarse depth bins so that the prefix surely fits the phase-1 capacity; no
// global depth sort is needed -- each tile's prefix list is depth-sorted on its own (k_tile_dsort).
// ---------------------------------------------------------------------------------------------------
constexpr int DH_THREADS = 256;
#ifndef DG_DH_ITEMS
#define DG_DH_ITEMS 32
#endif
constexpr int DH_ITEMS = DG_DH_ITEMS;               // Gaussians per thread per block
constexpr uint32_t DH_BASE = 0x3E4CCCCDu >> DH_SHIFT;  // bin of the near plane z = 0.2 (every visible key is above)

__device__ __forceinline__ uint32_t depth_bin(uint32_t key) {
    const uint32_t b = (key >> DH_SHIFT) - DH_BASE;
    return b < (uint32_t)DH_BINS ? b : (uint32_t)(DH_BINS - 1);  // far keys share the last bin
}

// hist[bin] += rect area of g over visible Gaussians: a private LDS histogram per block, flushed with one atomic per
// non-empty bin (blocks cover DH_THREADS * DH_ITEMS Gaussians: ~123 blocks at 1e6; 32 items per thread measured
// 0.7-0.9 us faster than 16 and 64 slower, profiles/r05an_depth_hist_ab.txt).
__global__ void __launch_bounds__(DH_THREADS) k_depth_hist(int P, const uint32_t* __restrict__ dkey,
                                                          const uint32_t* __restrict__ cnt,
                                                          uint32_t* __restrict__ hist) {
    __shared__ uint32_t s_h[DH_BINS];
    for (int i = threadIdx.x; i < DH_BINS; i += DH_THREADS) s_h[i] = 0u;
    __syncthreads();
    const int base = blockIdx.x * DH_THREADS * DH_ITEMS;
    uint32_t key[DH_ITEMS], c[DH_ITEMS];
#pragma unroll
    for (int k = 0; k < DH_ITEMS; k++) {  // every load in flight before the first use
        const int g = base + k * DH_THREADS + (int)threadIdx.x;
        key[k] = g < P ? dkey[g] : 0xffffffffu;
        c[k] = g < P ? cnt[g] : 0u;
    }
#pragma unroll
    for (int k = 0; k < DH_ITEMS; k++)
        if (key[k] != 0xffffffffu && c[k]) atomicAdd(&s_h[depth_bin(key[k])], c[k]);
    __syncthreads();
    for (int i = threadIdx.x; i < DH_BINS; i += DH_THREADS)
        if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

// One block: K = total rect area, and the largest bin prefix [0, b] whose rect areas fit `cap`; thr = the first
// key of bin b + 1 (S = {key < thr}).  No cut (thr = all visible) when K <= cap.  Also resets the per-view
// counters and the per-tile counters of both binning phases.
__device__ __forceinline__ void depth_cut_block(const uint32_t* __restrict__ hist, uint32_t cap,
                                                uint32_t* __restrict__ counters, uint32_t* __restrict__ tile_cnt,
                                                uint32_t* __restrict__ tile_cnt2, uint32_t num_tiles,
                                                const unsigned long long* __restrict__ rect_part, uint32_t nparts,
                                                uint32_t* __restrict__ probe);
__global__ void __launch_bounds__(1024) k_depth_cut(const uint32_t* __restrict__ hist, uint32_t cap,
                                                    uint32_t* __restrict__ counters, uint32_t* __restrict__ tile_cnt,
                                                    uint32_t* __restrict__ tile_cnt2, uint32_t num_tiles,
                                                    const unsigned long long* __restrict__ rect_part,
                                                    uint32_t nparts, uint32_t* __restrict__ probe) {
    depth_cut_block(hist, cap, counters, tile_cnt, tile_cnt2, num_tiles, rect_part, nparts, probe);
}

__device__ __forceinline__ void depth_cut_block(const uint32_t* __restrict__ hist, uint32_t cap,
                                                uint32_t* __restrict__ counters, uint32_t* __restrict__ tile_cnt,
                                                uint32_t* __restrict__ tile_cnt2, uint32_t num_tiles,
                                                const unsigned long long* __restrict__ rect_part, uint32_t nparts,
                                                uint32_t* __restrict__ probe) {
    __shared__ uint32_t s_w[16];
    __shared__ int s_best;
    __shared__ unsigned long long s_rect[16];
    __shared__ uint32_t s_err;
    constexpr int PER = DH_BINS / 1024;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // the histogram's loads go out first: the rect-area reduction and the zero fill below run under them
    uint32_t v[PER], loc = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) v[k] = hist[t * PER + k];
    if (t == 0) s_err = 0u;
    __syncthreads();
    {  // num_rendered = sum of the preprocess's per-block rect areas
        unsigned long long r = 0;
        bool e = false;
        // four parts per thread per round, loaded together (a 1e6 view has ~3.9k parts: one round trip, not four)
        for (uint32_t i0 = t; i0 < nparts; i0 += 4096) {
            unsigned long long pv[4];
#pragma unroll
            for (int k = 0; k < 4; k++) pv[k] = i0 + 1024u * k < nparts ? rect_part[i0 + 1024u * k] : 0ull;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                r += pv[k] & ~(1ull << 63);
                e |= (pv[k] >> 63) != 0ull;
            }
        }
        if (__any(e) && lane == 0) s_err = 1u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
        if (lane == 0) s_rect[w] = r;
    }
    for (uint32_t i = t; i < num_tiles; i += 1024) { tile_cnt[i] = 0u; tile_cnt2[i] = 0u; }
    // tile_cnt2 is followed by the replay-order histogram of the phase-2 launches (order_hist_piece: counts, cursors)
    for (uint32_t i = t; i < 2u * ORDER_NB; i += 1024) tile_cnt2[num_tiles + i] = 0u;
    if (t == 0) s_best = -1;
#pragma unroll
    for (int k = 0; k < PER; k++) loc += v[k];
    const uint32_t x = wave_incl_scan(loc);
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t off = 0, K = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) { if (k < w) off += s_w[k]; K += s_w[k]; }
    // inclusive cumulative count at each of this thread's bins; C(b) is non-decreasing in b
    uint32_t c = off + x - loc;
    int best = -1;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        c += v[k];
        if (c <= cap) best = t * PER + k;
    }
    if (best >= 0) atomicMax(&s_best, best);
    __syncthreads();
    if (t == 0) {
        unsigned long long r = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) r += s_rect[k];
        counters[CNT_RECT_LO] = (uint32_t)r;
        counters[CNT_RECT_LO + 1] = (uint32_t)(r >> 32);
        counters[CNT_ERR] = s_err;
        counters[CNT_INVD] = 0u; counters[10] = 0u; counters[13] = 0u;
        counters[CNT_PREV_UNF] = probe ? probe[0] : 0u;
        counters[CNT_PREV_K2] = probe ? probe[1] : 0u;
        if (probe) { probe[0] = 0u; probe[1] = 0u; }
    }
    const bool cut = K > cap;
    if (t == 0 && s_best < 0) {  // not even bin 0 fits: phase 1 bins nothing, phase 2 everything
        counters[CNT_K] = K;
        counters[CNT_THR] = cut ? (DH_BASE << DH_SHIFT) : 0xffffffffu;
        counters[CNT_E1] = 0u;  // accumulated by the emission
        counters[CNT_CUT] = cut ? 1u : 0u;
        counters[CNT_UNFINISHED] = 0; counters[CNT_K2] = 0; counters[CNT_LONG] = 0; counters[CNT_LONG2] = 0;
    }
    if (best >= 0 && best == s_best) {  // exactly one thread holds the best bin
        counters[CNT_K] = K;
        counters[CNT_THR] = cut ? ((DH_BASE + (uint32_t)best + 1u) << DH_SHIFT) : 0xffffffffu;
        counters[CNT_E1] = 0u;  // accumulated by the emission
        counters[CNT_CUT] = cut ? 1u : 0u;
        counters[CNT_UNFINISHED] = 0; counters[CNT_K2] = 0; counters[CNT_LONG] = 0; counters[CNT_LONG2] = 0;
    }
}


// Precise per-tile count of each lane's Gaussian (duplicateWithKeys' cull, rasterizer_impl.cu:149-179) by the
// wave-cooperative candidate walk, into cnt[lane] (LDS, zeroed here).  keep(tx, ty) filters tiles further.
template <typename Keep, typename OnKept>
__device__ __forceinline__ void wave_count(CandLDS& L, uint32_t* cnt, int lane, int x0, int y0, int x1, int y1,
                                           float mx, float my, float4 co, float thr, Keep&& keep, OnKept&& on_kept,
                                           uint64_t* kmask = nullptr) {
    cnt[lane] = 0u;
    wave_candidates(L, lane, x0, y0, x1, y1, mx, my, co, thr,
                    [&](int owner, int tx, int ty, bool kept, bool valid, uint32_t item) {
                        kept = kept && keep(tx, ty);
                        if (kept) on_kept(tx, ty);
                        const uint64_t km = __ballot(kept);
                        const uint32_t step = (item - (uint32_t)lane) >> 6;
                        if (kmask && lane == 0 && step < (uint32_t)KM_STEPS) kmask[step] = km;
                        // first item of each owner segment in this step adds the segment's kept count
                        const bool seg_start = valid && (lane == 0 || item == L.pre[owner]);
                        if (seg_start) {
                            const uint32_t seg_end_item = L.pre[owner] + (uint32_t)L.area[owner];
                            const int len = (int)min(seg_end_item - item, (uint32_t)(64 - lane));
                            const uint64_t seg = (len >= 64 ? ~0ull : ((1ull << len) - 1ull)) << lane;
                            cnt[owner] += (uint32_t)__popcll(km & seg);
                        }
                        __builtin_amdgcn_wave_barrier();
                    });
}

#ifndef DG_EMIT_RANKS
#define DG_EMIT_RANKS 64
#endif
constexpr int EMIT_RANKS = DG_EMIT_RANKS;  // Gaussians per wave of the binning walks

__device__ __forceinline__ uint32_t sat_rect(const uint32_t* sat, int tx, int x0, int y0, int x1, int y1);
// does the tile rect [x0,x1) x [y0,y1) hold an unfinished tile.  Layout of unf_rows (rw = words per tile row, th =
// tile rows): [th * rw] per-row bitmasks, [rw] their OR over all rows (columns holding an unfinished tile), [(th + 63)
// / 64] rows holding one.  The two summaries reject most rects with a load or two (every lane of a wave reads the same
// few words); the rows are walked four at a time only for rects that pass both.
__device__ __forceinline__ unsigned long long bits_range(int lo, int hi, int w) {  // bits [lo, hi) within word w
    const int a = lo - 64 * w > 0 ? lo - 64 * w : 0, b = hi - 64 * w < 64 ? hi - 64 * w : 64;
    if (b <= a) return 0ull;
    return (b == 64 ? ~0ull : ((1ull << b) - 1ull)) & ~((1ull << a) - 1ull);
}
__device__ __forceinline__ bool rows_touch(const BinArgs& a, int x0, int y0, int x1, int y1) {
    const int w0 = x0 >> 6, w1 = (x1 - 1) >> 6;
    const unsigned long long* cols = a.unf_rows + (size_t)a.unf_th * a.unf_rw;
    const unsigned long long* rany = cols + a.unf_rw;
    bool c = false, r = false;
    for (int w = w0; w <= w1; w++) c |= (cols[w] & bits_range(x0, x1, w)) != 0ull;
    for (int w = y0 >> 6; w <= (y1 - 1) >> 6; w++) r |= (rany[w] & bits_range(y0, y1, w)) != 0ull;
    if (!(c && r)) return false;
    for (int w = w0; w <= w1; w++) {
        const unsigned long long m = bits_range(x0, x1, w);
        for (int y = y0; y < y1; y += 4) {
            unsigned long long v = 0;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (y + k < y1) v |= a.unf_rows[(size_t)(y + k) * a.unf_rw + w];
            if (v & m) return true;
        }
    }
    return false;
}

// The binned Gaussians of a wave (EMIT_RANKS consecutive indices) and their walk inputs.
//   phase 1: the prefix Gaussians (key < thr);
//   phase 2: Gaussians past the threshold whose rect touches a tile phase 1 left unfinished (only those tiles kept).
struct BinLane {
    int x0, y0, x1, y1;
    float mx, my, lthr;
    float4 co;
    bool member;
};
// The walk's candidate tiles (DG_FULL_RECT_WALK: the whole rect): the rect's tiles that can meet the Gaussian's
// contribution ellipse E = {d : 0.5 d^T C d <= lthr} (alpha >= 1/255 at d; C = conic).  max_contrib_power_rect's kept
// test evaluates the power at a point of the tile's pixel rectangle, so a kept tile's rectangle holds a point of E and
// meets E's bounding box, half-widths sqrt(2 lthr Sigma_xx) and sqrt(2 lthr Sigma_yy), Sigma = C^-1 (det in double:
// no cancellation for thin conics; widened by 0.1% + 1 px against the test's float rounding).  The kept tiles, their
// count and their (ty, tx) order are those of the full rect: the walk only skips candidates the test rejects (the
// getRect radius is 3 sigma of the largest axis whatever the opacity and the orientation).
__device__ __forceinline__ void tight_rect(BinLane& b) {
#ifndef DG_FULL_RECT_WALK
    const double a_ = b.co.x, bb = b.co.y, c_ = b.co.z;
    const double det = a_ * c_ - bb * bb;
    if (!(det > 0.0) || !(a_ > 0.0) || !(c_ > 0.0)) return;  // degenerate conic (or NaN): the full rect
    const double L2 = 2.0 * (b.lthr > 0.0f ? (double)b.lthr : 0.0);
    const float wx = (float)sqrt(L2 * (c_ / det)) * 1.001f + 1.0f;
    const float wy = (float)sqrt(L2 * (a_ / det)) * 1.001f + 1.0f;
    // tiles t with [16 t, 16 t + 15] meeting [m - w, m + w]; clamped to the rect (fmaxf / fminf drop a NaN bound)
    const float fx0 = (float)b.x0, fx1 = (float)b.x1, fy0 = (float)b.y0, fy1 = (float)b.y1;
    const float lx = fminf(fmaxf(ceilf((b.mx - wx - (float)(GS_TILE_X - 1)) / (float)GS_TILE_X), fx0), fx1);
    const float hx = fminf(fmaxf(floorf((b.mx + wx) / (float)GS_TILE_X) + 1.0f, fx0), fx1);
    const float ly = fminf(fmaxf(ceilf((b.my - wy - (float)(GS_TILE_Y - 1)) / (float)GS_TILE_Y), fy0), fy1);
    const float hy = fminf(fmaxf(floorf((b.my + wy) / (float)GS_TILE_Y) + 1.0f, fy0), fy1);
    b.x0 = (int)lx; b.x1 = (int)hx; b.y0 = (int)ly; b.y1 = (int)hy;
    if (b.x1 < b.x0) b.x1 = b.x0;
    if (b.y1 < b.y0) b.y1 = b.y0;
#endif
}

// known: membership from the count pass's wave mask (0 / 1: no key test, no SAT test), -1: test here
template <int PHASE>
__device__ __forceinline__ BinLane bin_lane(const BinArgs& a, int g, int lane, uint32_t thr, uint32_t* s_key,
                                            int known = -1) {
    BinLane b = {0, 0, 0, 0, 0.f, 0.f, 0.f, make_float4(0.f, 0.f, 0.f, 0.f), false};
    if (lane < EMIT_RANKS && g < a.P && known != 0) {
        // phase 2's membership pass loads the rect half of the record together with the key (~95% of the Gaussians are
        // past the threshold and need it): one memory round trip fewer in the chain key -> rect -> unfinished rows
        const bool rect_first = PHASE == 2 && known < 0;
        float4 s1 = rect_first ? a.sp[2 * g + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
        const uint32_t key = a.dkey[g];
        s_key[lane] = key;
        bool m = known == 1 || (key != 0xffffffffu && (PHASE == 1 ? key < thr : key >= thr));
        if (m) {
            // phase 2 tests membership on the rect half of the record first: most past-threshold Gaussians touch no
            // unfinished tile, so only the members load the other 16 bytes
            float4 s0 = rect_first ? make_float4(0.f, 0.f, 0.f, 0.f) : a.sp[2 * g];
            if (!rect_first) s1 = a.sp[2 * g + 1];
            sp_rect(s1, b.x0, b.y0, b.x1, b.y1);
#ifdef DG_PHASE2_SAT
            if (PHASE == 2 && known < 0)
                m = b.x1 > b.x0 && b.y1 > b.y0 && sat_rect(a.sat, a.tiles_x, b.x0, b.y0, b.x1, b.y1) != 0u;
#else
            if (PHASE == 2 && known < 0) m = b.x1 > b.x0 && b.y1 > b.y0 && rows_touch(a, b.x0, b.y0, b.x1, b.y1);
#endif
            if (m && rect_first) s0 = a.sp[2 * g];
            if (m) {
                b.co = make_float4(s0.z, s0.w, s1.x, s1.y);
                b.mx = s0.x; b.my = s0.y;
                b.lthr = gs_crlogf(b.co.w / (1.0f / 255.0f));
                tight_rect(b);
            }
        }
        b.member = m;
    }
    if (!b.member) { b.x1 = b.x0; b.y1 = b.y0; }
    return b;
}

// Pass 1 of the binning: each wave's precise per-tile counts (rcnt of its Gaussians), the wave total (wtot) and
// the per-tile instance counts (tile_cnt, atomics without return).
template <int PHASE>
__global__ void __launch_bounds__(256) k_bin_count(BinArgs a) {
    __shared__ CandLDS s_cand[4];
    __shared__ uint32_t s_key[4][64];
    __shared__ uint32_t s_cnt[4][64];
    if (PHASE == 2 && a.probe && blockIdx.x == 0 && threadIdx.x == 0) a.probe[0] = a.counters[CNT_UNFINISHED];
    if (PHASE == 2 && a.counters[CNT_UNFINISHED] == 0u) return;  // phase 1 finished every tile
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wave = blockIdx.x * 4 + w;
    const int g0 = wave * EMIT_RANKS;
    if (g0 >= a.P) return;  // whole wave (past the last one the scan reads)
    const int g = g0 + lane;
    const BinLane b = bin_lane<PHASE>(a, g, lane, a.counters[CNT_THR], s_key[w]);
    const uint64_t members = __ballot(b.member);
    if (lane == 0) a.wmask[wave] = members;  // the emission pass skips the membership tests
    uint32_t c = 0;
    if (members) {
        wave_count(s_cand[w], s_cnt[w], lane, b.x0, b.y0, b.x1, b.y1, b.mx, b.my, b.co, b.lthr,
                   [&](int tx, int ty) { return PHASE == 1 || a.unf[ty * a.tiles_x + tx] != 0; },
                   [&](int tx, int ty) { atomicAdd(&a.tile_cnt[ty * a.tiles_x + tx], 1u); },
                   PHASE == 1 && KM_STEPS > 0 && a.kmask ? a.kmask + (size_t)wave * KM_STEPS : nullptr);
        c = s_cnt[w][lane];
        if (b.member) a.rcnt[g] = c;
    }
    const uint32_t tot = wave_sum_u32(c);
    if (lane == 0) a.wtot[wave] = tot;
}

// colour + inverse depth of a binned Gaussian (computeColorFromSH, forward.cu:24-76; 1 / view z)
__device__ __forceinline__ void binned_colour(const BinArgs& a, int g, uint32_t key) {
    f3 col;
    if (a.colors) {
        col = {a.colors[3 * g], a.colors[3 * g + 1], a.colors[3 * g + 2]};
    } else {
        const f3 po = {a.means3D[3 * g], a.means3D[3 * g + 1], a.means3D[3 * g + 2]};
        const f3 d0 = {a.dc[3 * g], a.dc[3 * g + 1], a.dc[3 * g + 2]};
        col = sh_to_rgb(po, a.campos, a.sh ? a.D : 0, d0, a.sh ? a.sh + (size_t)g * a.M * 3 : nullptr, nullptr);
    }
    a.rgbi[g] = make_float4(col.x, col.y, col.z, 1.f / __uint_as_float(key));
}

// colors_later: the phase-1 members that got instances, a Gaussian per lane (the emission's colour, launched after
// the overlapped SH update it reads)
__global__ void __launch_bounds__(256) k_binned_colors(BinArgs a) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= a.P || a.rcnt[g] == 0u) return;
    const uint32_t key = a.dkey[g];
    if (key == 0xffffffffu || key >= a.counters[CNT_THR]) return;  // phase 2's members get theirs from emit<2>
    binned_colour(a, g, key);
}

// The backward's replay length of a tile as the phase-2 launches see it: a finished tile's phase-1 max contributor
// (final), an unfinished tile's phase-1 + phase-2 list lengths (its max contributor is written by k_render_fwd2).
__device__ __forceinline__ uint32_t fwd2_replay_len(const uint8_t* unf, const uint32_t* max_contrib, const uint2* ranges1,
                                                    const uint2* ranges2, int tile) {
    if (!unf[tile]) return max_contrib[tile];
    const uint2 r1 = ranges1[tile], r2 = ranges2[tile];
    return (r1.y - r1.x) + (r2.y - r2.x);
}

__device__ __forceinline__ BinLane member_lane(const BinArgs& a, int g, bool member);

// Pass 2: wave base = exclusive scan of the wave totals (wtot, scanned in place); first_e of every binned
// Gaussian, and a second walk writes its instances (Gaussian, depth key) at consecutive indices in (lane, ty, tx)
// order, so every Gaussian's instances are contiguous: [first_e, first_e + rcnt); each instance index is also
// placed in its tile's list, s_e[atomic arrival cursor, from ranges[t].x] (counting sort; the order inside a tile is
// fixed afterwards by k_tile_dsort).
template <int PHASE>
__global__ void __launch_bounds__(256) k_bin_emit(BinArgs a) {
    __shared__ CandLDS s_cand[4];
    __shared__ uint32_t s_key[4][64];
    int bid = (int)blockIdx.x;
    if (PHASE == 2 && a.unf_sorted) {  // front block: the phase-2 tiles, longest list first (not gated)
        if (bid == 0) {
            const uint32_t nu = a.counters[CNT_UNFINISHED];
            uint32_t* cnt = &s_key[0][0];  // 256 buckets of (list length / 4), longest first
            if (threadIdx.x < 256) cnt[threadIdx.x] = 0u;
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < nu; i += 256) {
                const uint2 r = a.ranges[a.unf_list[i]];
                if (r.y > r.x) atomicAdd(&cnt[order_bucket(r.y - r.x)], 1u);
            }
            __syncthreads();
            {   // exclusive prefix of the 256 buckets: a wave scan per 64 + the wave totals (a serial loop over the
                // buckets by one thread was a ~10 us dependent LDS chain on this launch's critical path)
                __shared__ uint32_t wsum[4];
                const int t = threadIdx.x, ln = t & 63;
                const uint32_t v = cnt[t];
                uint32_t incl = v;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o);
                    if (ln >= o) incl += y;
                }
                if (ln == 63) wsum[t >> 6] = incl;
                __syncthreads();
                const uint32_t off = (t >= 64 ? wsum[0] : 0u) + (t >= 128 ? wsum[1] : 0u) + (t >= 192 ? wsum[2] : 0u);
                cnt[t] = off + incl - v;
                if (t == 255) const_cast<uint32_t*>(a.counters)[CNT_UNF2] = off + incl;
            }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < nu; i += 256) {
                const uint32_t tile = a.unf_list[i];
                const uint2 r = a.ranges[tile];
                if (r.y > r.x) a.unf_sorted[atomicAdd(&cnt[order_bucket(r.y - r.x)], 1u)] = tile;
            }
            return;
        }
        bid -= 1;
    }
    if (PHASE == 2 && a.ohist) {  // front blocks: the replay-order histogram (not gated: the backward needs the order)
        const int ob = order_blocks(a.num_tiles);
        if (bid < ob) {
            order_hist_piece(a.num_tiles, bid, a.ohist, &s_key[0][0], [&](int tile) {
                return fwd2_replay_len(a.unf, a.max_contrib, a.ranges1, a.ranges, tile);
            });
            return;
        }
        bid -= ob;
    }
    if (PHASE == 2 && a.counters[CNT_UNFINISHED] == 0u) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wave = bid * 4 + w;
    const int g0 = wave * EMIT_RANKS;
    if (g0 >= a.P) return;
    const uint64_t members = a.wmask[wave];
    if (!members) return;  // no member in this wave (no key, record or SAT loads)
    const int g = g0 + lane;
    // the count pass's members (each with g < P): key, record, count and the wave's base in one load round (bin_lane's
    // membership tests would put the key load in front of the others)
    const bool mine = lane < EMIT_RANKS && ((members >> lane) & 1ull) != 0ull;
    const uint32_t key = mine ? a.dkey[g] : 0u;
    const uint32_t base = a.wtot[wave];
    const uint32_t cm = mine ? a.rcnt[g] : 0u;
    const BinLane b = member_lane(a, g, mine);
    s_key[w][lane] = key;
    const uint32_t c = b.member ? cm : 0u;
    const uint32_t incl = wave_incl_scan(c);
    const uint32_t wt = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (wt == 0u || base + wt > a.cap) return;  // nothing kept; (capacity: never with consistent inputs)
    if (b.member && c) {
        a.first_e[g] = (PHASE == 2 ? a.counters[CNT_E1] : 0u) + base + incl - c;
        if (PHASE == 2 || !a.colors_later) binned_colour(a, g, s_key[w][lane]);
    }
    uint32_t running = 0;
    // phase 1: the kept ballots of the first KM_STEPS steps from the count pass (the same candidates, step by step)
    struct KnownKept {
        const uint64_t* km;
        __device__ __forceinline__ bool have(uint32_t step) const { return km && step < (uint32_t)KM_STEPS; }
        __device__ __forceinline__ uint64_t mask(uint32_t step) const { return km[step]; }
    };
    const KnownKept known = {PHASE == 1 && KM_STEPS > 0 && a.kmask ? a.kmask + (size_t)wave * KM_STEPS : nullptr};
    wave_candidates(s_cand[w], lane, b.x0, b.y0, b.x1, b.y1, b.mx, b.my, b.co, b.lthr,
                    [&](int owner, int tx, int ty, bool kept, bool, uint32_t) {
                        kept = kept && (PHASE == 1 || a.unf[ty * a.tiles_x + tx] != 0);
                        const uint64_t km = __ballot(kept);
                        const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
                        if (kept) {
                            const uint32_t e = base + running + (uint32_t)__popcll(km & lt);
                            const int t = ty * a.tiles_x + tx;
                            a.eg[e] = (uint32_t)(g0 + owner);
                            a.ikey[e] = s_key[w][owner];
                            a.flag[e] = 0;
                            a.s_e[atomicAdd(&a.tile_cnt[t], 1u)] = e;
                        }
                        running += (uint32_t)__popcll(km);
                    }, known);
}

// ---- Fat binning waves (R x 64 consecutive Gaussians per wave; DG_BIN_FAT1 / DG_BIN_FAT2 = R of phase 1 / 2).
// Most Gaussians of a wave are not members (phase 1: ~5% are in front of the threshold; phase 2: only those whose
// rect touches an unfinished tile), so a 64-Gaussian wave mostly tests and exits, and its memory round trips are the
// cost.  A fat wave loads the keys (and, in phase 2, the rect halves) of all R x 64 Gaussians at once, compacts its
// members in LDS (index order), walks them 64 at a time and hands the member list to the emission pass, which then
// skips every membership test.  The members stay in index order, so the emission numbering -- and every output -- is
// the one of the 64-Gaussian waves.
#ifndef DG_BIN_FAT1
#define DG_BIN_FAT1 1
#endif
#ifndef DG_BIN_FAT2
#define DG_BIN_FAT2 1
#endif
template <int PHASE> struct FatR { static constexpr int R = PHASE == 1 ? DG_BIN_FAT1 : DG_BIN_FAT2; };
template <int PHASE> __host__ __device__ constexpr int fat_span() { return 64 * FatR<PHASE>::R; }

// walk inputs of a known member g (BinLane with the membership already decided)
__device__ __forceinline__ BinLane member_lane(const BinArgs& a, int g, bool member) {
    BinLane b = {0, 0, 0, 0, 0.f, 0.f, 0.f, make_float4(0.f, 0.f, 0.f, 0.f), false};
    if (member) {
        const float4 s0 = a.sp[2 * g], s1 = a.sp[2 * g + 1];
        sp_rect(s1, b.x0, b.y0, b.x1, b.y1);
        b.co = make_float4(s0.z, s0.w, s1.x, s1.y);
        b.mx = s0.x; b.my = s0.y;
        b.lthr = gs_crlogf(b.co.w / (1.0f / 255.0f));
        tight_rect(b);
        b.member = true;
    }
    if (!b.member) { b.x1 = b.x0; b.y1 = b.y0; }
    return b;
}

template <int PHASE>
__global__ void __launch_bounds__(256) k_bin_count_fat(BinArgs a) {
    constexpr int R = FatR<PHASE>::R, S = 64 * R;
    __shared__ CandLDS s_cand[4];
    __shared__ uint32_t s_cnt[4][64];
    __shared__ uint32_t s_mem[4][S];
    if (PHASE == 2 && a.probe && blockIdx.x == 0 && threadIdx.x == 0) a.probe[0] = a.counters[CNT_UNFINISHED];
    if (PHASE == 2 && a.counters[CNT_UNFINISHED] == 0u) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wave = blockIdx.x * 4 + w;
    const int g0 = wave * S;
    if (g0 >= a.P) return;
    const uint32_t thr = a.counters[CNT_THR];
    uint32_t key[R];
#pragma unroll
    for (int r = 0; r < R; r++) {  // every key load in flight at once
        const int g = g0 + 64 * r + lane;
        key[r] = g < a.P ? a.dkey[g] : 0xffffffffu;
    }
    bool mem[R];
    if (PHASE == 1) {
#pragma unroll
        for (int r = 0; r < R; r++) mem[r] = key[r] != 0xffffffffu && key[r] < thr;
    } else {
        float4 s1[R];
#pragma unroll
        for (int r = 0; r < R; r++) {  // the rect halves of the past-threshold Gaussians, all at once
            const bool c = key[r] != 0xffffffffu && key[r] >= thr;
            s1[r] = c ? a.sp[2 * (g0 + 64 * r + lane) + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
            mem[r] = c;
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (!mem[r]) continue;
            int x0, y0, x1, y1;
            sp_rect(s1[r], x0, y0, x1, y1);
            mem[r] = x1 > x0 && y1 > y0 && rows_touch(a, x0, y0, x1, y1);
        }
    }
    // compact the members (index order) into LDS and the wave's slice of the global member list
    uint32_t nm = 0;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint64_t bm = __ballot(mem[r]);
        if (mem[r]) {
            const uint32_t slot = nm + (uint32_t)__popcll(bm & lt);
            s_mem[w][slot] = (uint32_t)(64 * r + lane);
            a.mlist[g0 + slot] = (uint32_t)(64 * r + lane);
        }
        nm += (uint32_t)__popcll(bm);
    }
    if (lane == 0) a.wmask[wave] = nm;
    __builtin_amdgcn_wave_barrier();
    uint32_t tot = 0;
    for (uint32_t mb = 0; mb < nm; mb += 64) {
        const uint32_t i = mb + (uint32_t)lane;
        const bool member = i < nm;
        const int g = member ? g0 + (int)s_mem[w][i] : 0;
        const BinLane b = member_lane(a, g, member);
        wave_count(s_cand[w], s_cnt[w], lane, b.x0, b.y0, b.x1, b.y1, b.mx, b.my, b.co, b.lthr,
                   [&](int tx, int ty) { return PHASE == 1 || a.unf[ty * a.tiles_x + tx] != 0; },
                   [&](int tx, int ty) { atomicAdd(&a.tile_cnt[ty * a.tiles_x + tx], 1u); },
                   PHASE == 1 && KM_STEPS > 0 && a.kmask ? a.kmask + (size_t)wave * KM_STEPS : nullptr);
        const uint32_t c = member ? s_cnt[w][lane] : 0u;
        if (member) a.rcnt[g] = c;
        uint32_t sc = c;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sc += __shfl_xor(sc, o);
        tot += sc;
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) a.wtot[wave] = tot;
}

template <int PHASE>
__global__ void __launch_bounds__(256) k_bin_emit_fat(BinArgs a) {
    constexpr int S = fat_span<PHASE>();
    __shared__ CandLDS s_cand[4];
    __shared__ uint32_t s_key[4][64];
    __shared__ uint32_t s_g[4][64];
    if (PHASE == 2 && a.counters[CNT_UNFINISHED] == 0u) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wave = blockIdx.x * 4 + w;
    const int g0 = wave * S;
    if (g0 >= a.P) return;
    const uint32_t nm = (uint32_t)a.wmask[wave];
    if (!nm) return;
    const uint32_t base = a.wtot[wave];
    const uint32_t e_off = PHASE == 2 ? a.counters[CNT_E1] : 0u;
    uint32_t running = 0;
    for (uint32_t mb = 0; mb < nm; mb += 64) {
        const uint32_t i = mb + (uint32_t)lane;
        const bool member = i < nm;
        const int g = member ? g0 + (int)a.mlist[g0 + i] : 0;
        const uint32_t key = member ? a.dkey[g] : 0u;
        s_key[w][lane] = key;
        s_g[w][lane] = (uint32_t)g;
        const BinLane b = member_lane(a, g, member);
        const uint32_t c = member ? a.rcnt[g] : 0u;
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t wt = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (base + running + wt > a.cap) return;  // (capacity: never with consistent inputs)
        if (member && c) {
            a.first_e[g] = e_off + base + running + incl - c;
            if (PHASE == 2 || !a.colors_later) binned_colour(a, g, key);
        }
        __builtin_amdgcn_wave_barrier();
        if (wt) {
            uint32_t run = running;
            wave_candidates(s_cand[w], lane, b.x0, b.y0, b.x1, b.y1, b.mx, b.my, b.co, b.lthr,
                            [&](int owner, int tx, int ty, bool kept, bool, uint32_t) {
                                kept = kept && (PHASE == 1 || a.unf[ty * a.tiles_x + tx] != 0);
                                const uint64_t km = __ballot(kept);
                                const uint64_t ltm = lane == 0 ? 0ull : (~0ull >> (64 - lane));
                                if (kept) {
                                    const uint32_t e = base + run + (uint32_t)__popcll(km & ltm);
                                    const int t = ty * a.tiles_x + tx;
                                    a.eg[e] = s_g[w][owner];
                                    a.ikey[e] = s_key[w][owner];
                                    a.flag[e] = 0;
                                    a.s_e[atomicAdd(&a.tile_cnt[t], 1u)] = e;
                                }
                                run += (uint32_t)__popcll(km);
                            });
        }
        running += wt;
        __builtin_amdgcn_wave_barrier();
    }
}

// Exclusive summed-area table of the unfinished-tile flags, [(tiles_y+1) x (tiles_x+1)]: O(1) "does this
// rect touch an unfinished tile" for the phase-2 kernels.  Two wave-parallel passes (one wave per row, then one
// per column, 64-wide shuffle scans), so no lane walks a dependent chain of global accesses.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}
__global__ void __launch_bounds__(256) k_sat_rows(const uint32_t* __restrict__ counters,
                                                  const uint8_t* __restrict__ unf, int tx, int ty,
                                                  uint32_t* __restrict__ sat, uint32_t* __restrict__ probe) {
    if (probe && blockIdx.x == 0 && threadIdx.x == 0) *probe = counters[CNT_UNFINISHED];
    if (counters[CNT_UNFINISHED] == 0u) return;
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);  // sat row r = tile row r - 1
    if (r > ty) return;
    const int W1 = tx + 1;
    uint32_t* row = sat + (size_t)r * W1;
    if (lane == 0) row[0] = 0u;
    uint32_t carry = 0u;
    for (int x0 = 0; x0 < tx; x0 += 64) {
        const int x = x0 + lane;
        const uint32_t v = (r > 0 && x < tx && unf[(size_t)(r - 1) * tx + x]) ? 1u : 0u;
        const uint32_t inc = wave_incl_scan(v, lane) + carry;
        if (x < tx) row[x + 1] = inc;
        carry = __shfl(inc, 63);
    }
}
__global__ void __launch_bounds__(256) k_sat_cols(const uint32_t* __restrict__ counters, int tx, int ty,
                                                  uint32_t* __restrict__ sat) {
    if (counters[CNT_UNFINISHED] == 0u) return;
    const int lane = threadIdx.x & 63, c = 1 + blockIdx.x * 4 + (threadIdx.x >> 6);  // column 0 is all zero
    if (c > tx) return;
    const int W1 = tx + 1;
    uint32_t carry = 0u;
    for (int y0 = 1; y0 <= ty; y0 += 64) {
        const int y = y0 + lane;
        const uint32_t v = y <= ty ? sat[(size_t)y * W1 + c] : 0u;
        const uint32_t inc = wave_incl_scan(v, lane) + carry;
        if (y <= ty) sat[(size_t)y * W1 + c] = inc;
        carry = __shfl(inc, 63);
    }
}

__device__ __forceinline__ uint32_t sat_rect(const uint32_t* sat, int tx, int x0, int y0, int x1, int y1) {
    const int W1 = tx + 1;
    return sat[(size_t)y1 * W1 + x1] - sat[(size_t)y0 * W1 + x1] - sat[(size_t)y1 * W1 + x0] + sat[(size_t)y0 * W1 + x0];
}

__device__ __forceinline__ float bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ uint32_t bcast_u(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

// renderCUDA (forward.cu:349-501) restructured for wave64: one wave per 16x16 tile, 4 pixels per lane.
// Lane l owns pixels (l&7, l>>3) and (l&7 + 8, l>>3) of the top half (pair A = quadrants 0,1) and the
// same two of the bottom half (pair B = quadrants 2,3); each pair is one row, evaluated with packed fp32.
// Each 64-splat batch is gathered one splat per lane (one 32-B splat record + colour), tested against
// the four quadrants with the reference's own max-contribution rect test (quad_mask), and staged in
// wave-private LDS; the wave then walks only splats that reach a quadrant (s_ff1 over a 64-bit ballot),
// reads each with broadcast ds_read_b128 and skips a pair whose two quadrant bits are clear.  The
// per-pixel update is branch-free: a rejected or finished pixel gets alpha = 0, which leaves C, D and T
// unchanged.  Wave-uniform early exit once every pixel of the tile has saturated.
#ifndef DG_FWD_GROUP
#define DG_FWD_GROUP 4
#endif
constexpr int FWD_GROUP = DG_FWD_GROUP;  // splats per branch-free group of the compositing loop

#ifdef DG_FWD_WPE  // occupancy experiment: cap VGPRs so that DG_FWD_WPE waves fit per SIMD
#define FWD_WPE_ATTR __attribute__((amdgpu_waves_per_eu(DG_FWD_WPE)))
#else
#define FWD_WPE_ATTR
#endif
template <int PHASE, bool COUNT>
__global__ void __launch_bounds__(256) FWD_WPE_ATTR k_render_fwd(RenderArgs a) {
    // per wave: the sort's scratch (cnt 256 + keys 512 + values 512 u32), then 64 staged splats + a null splat
    // (opacity 0: no pixel accepts it) = 780 u32 and the sorted list (512 u32)
    constexpr int WAVE_LDS = 780 + DS_WAVE_MAX;
    __shared__ __attribute__((aligned(16))) uint32_t s_raw[4][WAVE_LDS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the counters the host waits for are final (written by the launches before this one): system-scope stores to the
    // coherent pinned buffer, then the sequence word behind a system-scope release
    if (PHASE == 1 && a.hc_dst && blockIdx.x == 0 && threadIdx.x == 0) {
        for (int i = 0; i < 16; i++)
            __hip_atomic_store(a.hc_dst + i, a.hc_src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.hc_dst + 16, a.hc_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const int tile = blockIdx.x * 4 + w;
    if (tile >= a.num_tiles) return;
    // the adaptive capacity's probe gets this view's phase-2 instance count (the next view's k_depth_cut reads it)
    if (PHASE == 2 && a.probe && blockIdx.x == 0 && threadIdx.x == 0) a.probe[1] = a.counters[CNT_K2];
    if (PHASE == 2 && !a.unfinished[tile]) return;  // finished in phase 1: outputs already final
    float4* sb = reinterpret_cast<float4*>(&s_raw[w][0]);
    uint32_t* ids = &s_raw[w][780];
    bool lds_ids = false;
    if (PHASE == 1 && a.fuse_sort) {
        const int ns = wave_sort_tile<DS_ROWS>(a.ds, tile, lane, &s_raw[w][0], &s_raw[w][256], &s_raw[w][768], ids);
        lds_ids = ns > 1 && ns <= DS_WAVE_MAX;  // 0/1 need no sort, longer lists were sorted before the render
    }
    if (lane < 3) sb[64 * 3 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int tx0 = tx * GS_TILE_X, ty0 = ty * GS_TILE_Y;
    const int c0 = tx0 + (lane & 7), rA = ty0 + (lane >> 3);
    const v4f pxv = {(float)c0, (float)c0, (float)(c0 + 8), (float)(c0 + 8)};
    const v2f pyv = {(float)rA, (float)(rA + 8)};
    // per-pixel state; a finished (or outside) pixel gets alpha threshold 2, which no alpha reaches
    v4f T = bc4(1.0f), C0 = bc4(0.0f), C1 = bc4(0.0f), C2 = bc4(0.0f), D = bc4(0.0f), thr;
    uint32_t last[4] = {0, 0, 0, 0};
    uint32_t cbase = 0;  // contributor numbering continues over the concatenated phase-1 + phase-2 list
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int px = c0 + (k >> 1) * 8, py = rA + (k & 1) * 8;
        const bool inside = px < a.W && py < a.H;
        thr[k] = inside ? (1.0f / 255.0f) : 2.0f;
        if (PHASE == 2 && inside) {  // resume the phase-1 state of this pixel
            const size_t pid = (size_t)py * a.W + px;
            const float4 rs = a.resume[pid];
            T[k] = a.final_T[pid];
            D[k] = a.img_invd[pid];
            last[k] = a.n_contrib[pid];
            C0[k] = rs.x; C1[k] = rs.y; C2[k] = rs.z; thr[k] = rs.w;
        }
    }
    if (PHASE == 2) cbase = a.ranges1[tile].y - a.ranges1[tile].x;
    const uint2 rg = a.ranges[tile];
    const int n = (int)(rg.y - rg.x);
    for (int base = 0; base < n; base += 64) {
        if (!__any(fminf(fminf(thr.x, thr.y), fminf(thr.z, thr.w)) < 1.0f)) break;
        const int j = base + lane;
        bool touch = false;
        if (j < n) {
            const uint32_t e = min(lds_ids ? ids[j] : a.s_e[rg.x + j], a.K - 1);
            const uint32_t g = min(a.eg[e], a.P - 1);
            const float4 s0 = a.sp[2 * g], s1 = a.sp[2 * g + 1];
            const float4 q = a.rgbi[g];
            const float lthr = quad_log_thr(s1.y);
            touch = quad_mask({s0.z, s0.w, s1.x, s1.y}, s0.x, s0.y, lthr, tx0, ty0) != 0u;
            const SplatExp k = splat_exp_coeffs(s0.z, s0.w, s1.x);
            sb[lane * 3 + 0] = make_float4(s0.x, s0.y, k.A, k.B);
            sb[lane * 3 + 1] = make_float4(k.C, s1.y, q.x, q.y);
            sb[lane * 3 + 2] = make_float4(q.z, q.w, __uint_as_float(g), 0.0f);
        }
        __builtin_amdgcn_wave_barrier();
        uint64_t mask = __ballot(touch);
        // Splats go in groups of FWD_GROUP with no branch between them (a group's missing tail is the null splat), and the
        // saturation exit is tested once per group: per-splat control flow costs more than the null splats do.
        while (mask) {
#ifdef DG_FWD_FAST
          // Two passes over the group: alphas first, then a wave-uniform test of whether any pixel's T can fall below
          // 1e-4 inside the group (T only falls, and the chained product is exactly the per-splat test_T sequence).
          // When none can, the group commits without the termination selects; otherwise the per-splat sequence runs.
          int jg[FWD_GROUP];
          v4f alg[FWD_GROUP];
          uint32_t accb[FWD_GROUP];
          v4f Tt = T;
#pragma unroll
          for (int u = 0; u < FWD_GROUP; u++) {
            const int jj = mask ? (int)__builtin_ctzll(mask) : 64;
            mask &= mask - 1;
            jg[u] = jj;
            const float4 Sa = sb[jj * 3 + 0], Sb = sb[jj * 3 + 1];
            const v4f p2 = splat_power4(Sa.z, Sa.w, Sb.x, Sa.x, Sa.y, pxv, pyv);
            v4f al = bc4(Sb.y) * (v4f){__builtin_amdgcn_exp2f(p2.x), __builtin_amdgcn_exp2f(p2.y),
                                       __builtin_amdgcn_exp2f(p2.z), __builtin_amdgcn_exp2f(p2.w)};
            uint32_t ab = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float ak = fminf(0.99f, al[k]);
                const bool ok = !(p2[k] > 0.0f || ak < thr[k]);
                al[k] = ok ? ak : 0.0f;
                ab |= ok ? (1u << k) : 0u;
            }
            alg[u] = al;
            accb[u] = ab;
            Tt = Tt * (bc4(1.0f) - al);
          }
          const bool safe = !COUNT && !__any(fminf(fminf(Tt.x, Tt.y), fminf(Tt.z, Tt.w)) < 0.0001f);
          if (safe) {
#pragma unroll
            for (int u = 0; u < FWD_GROUP; u++) {
              const float4 Sb = sb[jg[u] * 3 + 1], Sc = sb[jg[u] * 3 + 2];
              const uint32_t c = cbase + (uint32_t)(base + jg[u] + 1);
              const v4f wt = alg[u] * T;
              C0 = fma4(bc4(Sb.z), wt, C0);
              C1 = fma4(bc4(Sb.w), wt, C1);
              C2 = fma4(bc4(Sc.x), wt, C2);
              D = fma4(bc4(Sc.y), wt, D);
              T = T * (bc4(1.0f) - alg[u]);
#pragma unroll
              for (int k = 0; k < 4; k++) last[k] = (accb[u] >> k) & 1u ? c : last[k];
            }
          } else {
#pragma unroll
            for (int u = 0; u < FWD_GROUP; u++) {
              const float4 Sb = sb[jg[u] * 3 + 1], Sc = sb[jg[u] * 3 + 2];
              const uint32_t c = cbase + (uint32_t)(base + jg[u] + 1);
              v4f al = alg[u];
              const v4f test_T = T * (bc4(1.0f) - al);
              v4f Tn;
              bool acc[4];
#pragma unroll
              for (int k = 0; k < 4; k++) {
                  acc[k] = (accb[u] >> k) & 1u;
                  const bool term = test_T[k] < 0.0001f;
                  thr[k] = term ? 2.0f : thr[k];
                  al[k] = term ? 0.0f : al[k];
                  Tn[k] = term ? T[k] : test_T[k];
                  last[k] = (acc[k] && !term) ? c : last[k];
              }
              if (COUNT) {
                  uint32_t n = 0;
#pragma unroll
                  for (int k = 0; k < 4; k++) n += (uint32_t)__popcll(__ballot(acc[k] && al[k] != 0.0f));
                  if (n && lane == 0) atomicAdd(a.gcount + __float_as_uint(Sc.z), n);
              }
              const v4f wt = al * T;
              C0 = fma4(bc4(Sb.z), wt, C0);
              C1 = fma4(bc4(Sb.w), wt, C1);
              C2 = fma4(bc4(Sc.x), wt, C2);
              D = fma4(bc4(Sc.y), wt, D);
              T = Tn;
            }
          }
#else
          // TERM = false: the group cannot take any pixel's T below 1e-4, so the termination selects are dropped
          auto group = [&](auto term_c) {
          constexpr bool TERM = decltype(term_c)::value;
#pragma unroll
          for (int u = 0; u < FWD_GROUP; u++) {
            const int jj = mask ? (int)__builtin_ctzll(mask) : 64;
            mask &= mask - 1;
            const float4 Sa = sb[jj * 3 + 0], Sb = sb[jj * 3 + 1], Sc = sb[jj * 3 + 2];
            const uint32_t c = cbase + (uint32_t)(base + jj + 1);
            const v4f p2 = splat_power4(Sa.z, Sa.w, Sb.x, Sa.x, Sa.y, pxv, pyv);
            v4f al = bc4(Sb.y) * (v4f){__builtin_amdgcn_exp2f(p2.x), __builtin_amdgcn_exp2f(p2.y),
                                       __builtin_amdgcn_exp2f(p2.z), __builtin_amdgcn_exp2f(p2.w)};
            // forward.cu:451-475: skip power > 0 and alpha < 1/255, stop once T would fall below 1e-4
            bool acc[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float ak = fminf(0.99f, al[k]);
                acc[k] = !(p2[k] > 0.0f || ak < thr[k]);
                al[k] = acc[k] ? ak : 0.0f;
            }
            const v4f test_T = T * (bc4(1.0f) - al);
            v4f Tn;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool term = TERM && test_T[k] < 0.0001f;
                thr[k] = term ? 2.0f : thr[k];
                al[k] = term ? 0.0f : al[k];
                Tn[k] = term ? T[k] : test_T[k];
                last[k] = (acc[k] && !term) ? c : last[k];  // contributed: accepted and not the stopping splat
            }
            if (COUNT) {  // LightGaussian count mode: pixels the splat contributes to (old forward.cu:481-487)
                uint32_t n = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) n += (uint32_t)__popcll(__ballot(acc[k] && al[k] != 0.0f));
                if (n && lane == 0) atomicAdd(a.gcount + __float_as_uint(Sc.z), n);
            }
            const v4f wt = al * T;
            C0 = fma4(bc4(Sb.z), wt, C0);
            C1 = fma4(bc4(Sb.w), wt, C1);
            C2 = fma4(bc4(Sc.x), wt, C2);
            D = fma4(bc4(Sc.y), wt, D);
            T = Tn;
          }
          };
#ifdef DG_FWD_BOUND
          // Exact, wave-uniform bound: a splat's alpha is at most min(0.99, opacity), and rounded products and
          // differences are monotone, so the chain min_live(T) * prod(1 - min(0.99, opacity)) bounds every live
          // pixel's T after the group from below (margin 1.001 for the exp2 approximation at 0).  Finished pixels
          // (threshold 2) accept nothing and do not count.
          float tb = 1.0f;
#pragma unroll
          for (int k = 0; k < 4; k++) tb = fminf(tb, thr[k] < 1.0f ? T[k] : 1.0f);
          {
            uint64_t m2 = mask;
#pragma unroll
            for (int u = 0; u < FWD_GROUP; u++) {
              const int jj = m2 ? (int)__builtin_ctzll(m2) : 64;
              m2 &= m2 - 1;
              tb = tb * (1.0f - fminf(0.99f, sb[jj * 3 + 1].y));
            }
          }
          if (!COUNT && !__any(tb < 1.001e-4f)) group(std::false_type{});
          else group(std::true_type{});
#else
          group(std::true_type{});
#endif
#endif
            // early exit, checked every 8 splats (splats after saturation leave every pixel unchanged)
            if (!__any(fminf(fminf(thr.x, thr.y), fminf(thr.z, thr.w)) < 1.0f)) break;
        }
        __builtin_amdgcn_wave_barrier();
    }
    const size_t HW = (size_t)a.W * a.H;
    uint32_t mx = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int px = c0 + (k >> 1) * 8, py = rA + (k & 1) * 8;
        if (!(px < a.W && py < a.H)) continue;
        const size_t pid = (size_t)py * a.W + px;
        a.final_T[pid] = T[k];
        a.n_contrib[pid] = last[k];
        const float o0 = fmaf(T[k], a.bg[0], C0[k]);
        const float o1 = fmaf(T[k], a.bg[1], C1[k]);
        const float o2 = fmaf(T[k], a.bg[2], C2[k]);
        a.out_color[pid] = o0; a.out_color[HW + pid] = o1; a.out_color[2 * HW + pid] = o2;
        a.img_color[pid] = o0; a.img_color[HW + pid] = o1; a.img_color[2 * HW + pid] = o2;
        a.out_invd[pid] = D[k];
        a.img_invd[pid] = D[k];
        mx = last[k] > mx ? last[k] : mx;
    }
    mx = wave_max_u32(mx);
    if (lane == 0) a.max_contrib[tile] = mx;
    if (PHASE == 1) {
        // A tile with a live pixel after a truncated (prefix) list needs phase 2: keep its raw state.
        const bool cut = a.counters[CNT_CUT] != 0u;
        const bool live = fminf(fminf(thr.x, thr.y), fminf(thr.z, thr.w)) < 1.0f;
        const bool unf = cut && __any(live);
        if (lane == 0) {
            a.unfinished[tile] = unf ? 1 : 0;
            if (unf) {
                const uint32_t slot = atomicAdd(a.counters + CNT_UNFINISHED, 1u);
                if (a.unf_list) a.unf_list[slot] = (uint32_t)tile;
                a.ranges2_zero[tile] = make_uint2(0u, 0u);  // empty unless phase 2 bins instances for it
                if (a.unf_rows) {  // row word, column summary, row summary (rows_touch's layout)
                    const int th = (a.num_tiles + a.tiles_x - 1) / a.tiles_x;
                    atomicOr(a.unf_rows + (size_t)ty * a.unf_rw + (tx >> 6), 1ull << (tx & 63));
                    atomicOr(a.unf_rows + (size_t)th * a.unf_rw + (tx >> 6), 1ull << (tx & 63));
                    atomicOr(a.unf_rows + (size_t)(th + 1) * a.unf_rw + (ty >> 6), 1ull << (ty & 63));
                }
            }
        }
        if (unf) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int px = c0 + (k >> 1) * 8, py = rA + (k & 1) * 8;
                if (px < a.W && py < a.H) a.resume[(size_t)py * a.W + px] = make_float4(C0[k], C1[k], C2[k], thr[k]);
            }
        }
    }
}

// Phase 2 of renderCUDA (forward.cu:441-591 over the rest of the list) for the tiles phase 1 left unfinished: one
// 256-thread block per tile, one pixel per lane (wave w owns rows 4w..4w+3 of the tile).  These few tiles carry the
// view's longest phase-2 lists (typically tiles that see only splats past the depth threshold) and run nearly alone
// on the chip, so their latency is the cost: the block gathers the list in chunks of FWD2_CHUNK splats into LDS
// with every thread's loads in flight at once (one dependent-load chain per chunk instead of one per 64 splats of a
// lone wave), and each wave walks the chunk in branch-free groups of four splats (null-splat padding, as
// k_render_fwd) with one pixel per lane.  The per-pixel arithmetic is k_render_fwd's (splat_exp_coeffs, the
// splat_power4 operation order, the same accept / stop / update sequence), so the backward's replay reproduces
// every decision.  Every splat of the list is evaluated (the quadrant test only skips splats no pixel accepts).
#ifndef DG_FWD2_CHUNK
#define DG_FWD2_CHUNK 1024
#endif
constexpr int FWD2_CHUNK = DG_FWD2_CHUNK;
static_assert(FWD2_CHUNK >= 256 && FWD2_CHUNK % 64 == 0, "the chunk buffer is also the sorts' and the order's scratch");
template <bool COUNT>
__device__ __forceinline__ void render_fwd2_tile(const RenderArgs& a, int tile, float4* s_sb, uint32_t* s_mx,
                                                 uint32_t* s_ids);
constexpr int FWD2_GRID = 1024;  // blocks of the list-walking launch (a 1080p view has 0 to ~1100 unfinished tiles)
template <bool COUNT>
__global__ void __launch_bounds__(256) k_render_fwd2(RenderArgs a) {
    __shared__ __attribute__((aligned(16))) float4 s_sb[(FWD2_CHUNK + 4) * 3];  // (also the sort's scratch)
    __shared__ uint32_t s_mx[4];
    __shared__ uint32_t s_ids[DS_WAVE_MAX2];
    // the adaptive capacity's probe gets this view's phase-2 instance count (the next view's k_depth_cut reads it)
    if (a.probe && blockIdx.x == 0 && threadIdx.x == 0) a.probe[1] = a.counters[CNT_K2];
    // the front blocks (dispatched first, so they overlap the tiles' blocks): the backward's longest-first replay
    // order, scattered from the buckets the phase-2 emission histogrammed (order_scatter_piece; one block sorting every
    // tile without ohist) -- a finished tile's phase-1 max contributor is final, an unfinished tile's replay is bounded
    // by its phase-1 + phase-2 list lengths (max_contrib is read only where the other blocks do not write it)
    const uint32_t ob = a.order ? (a.ohist ? (uint32_t)order_blocks(a.num_tiles) : 1u) : 0u;
    if (blockIdx.x < ob) {
        const auto len = [&](int tile) { return fwd2_replay_len(a.unfinished, a.max_contrib, a.ranges1, a.ranges, tile); };
        if (a.ohist) {  // the emission's front blocks histogrammed the buckets
            uint32_t* scr = reinterpret_cast<uint32_t*>(s_sb);
            order_scatter_piece(a.num_tiles, (int)blockIdx.x, a.ohist, a.order, scr, scr + ORDER_NB, scr + 2 * ORDER_NB,
                                len);
        } else {
            tile_order_sort(a.num_tiles, a.order, len);
        }
        return;
    }
    if (a.unf_sorted) {  // the tiles with phase-2 instances, longest first, a block each, grid-stride
        const uint32_t nu = a.counters[CNT_UNF2];
        for (uint32_t i = blockIdx.x - ob; i < nu; i += gridDim.x - ob) {
            render_fwd2_tile<COUNT>(a, (int)a.unf_sorted[i], s_sb, s_mx, s_ids);
            __syncthreads();  // s_sb / s_ids are reused by the next tile
        }
        return;
    }
    if (a.unf_list) {  // the unfinished tiles phase 1 listed, a block each, grid-stride
        const uint32_t nu = a.counters[CNT_UNFINISHED];
        for (uint32_t i = blockIdx.x - ob; i < nu; i += gridDim.x - ob) {
            render_fwd2_tile<COUNT>(a, (int)a.unf_list[i], s_sb, s_mx, s_ids);
            __syncthreads();  // s_sb / s_ids are reused by the next tile
        }
        return;
    }
    const int tile = (int)(blockIdx.x - ob);
    if (tile >= a.num_tiles || !a.unfinished[tile]) return;  // block-uniform: finished in phase 1
    render_fwd2_tile<COUNT>(a, tile, s_sb, s_mx, s_ids);
}
template <bool COUNT>
__device__ __forceinline__ void render_fwd2_tile(const RenderArgs& a, int tile, float4* s_sb, uint32_t* s_mx,
                                                 uint32_t* s_ids) {
    const uint2 rg = a.ranges[tile];
    const int n = (int)(rg.y - rg.x);
    // No phase-2 instance (e.g. an image-edge tile whose list ended unsaturated in phase 1): phase 1 already wrote this
    // tile's final outputs (colour with the background, T, inverse depth, last contributors, max contributor) -- the
    // values this pass would rewrite -- so the block skips it.  Block-uniform.  (Two thirds of the unfinished tiles of
    // some yaw views; with more unfinished tiles than blocks they made blocks composite two tiles in a row.)
    if (n == 0) return;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int px = tx * GS_TILE_X + (lane & 15), py = ty * GS_TILE_Y + 4 * w + (lane >> 4);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;
    float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f, D = 0.0f, thr = 2.0f;
    uint32_t last = 0;
    const size_t pid = inside ? (size_t)py * a.W + px : 0;
    if (inside) {  // resume the phase-1 state of this pixel
        const float4 rs = a.resume[pid];
        T = a.final_T[pid];
        D = a.img_invd[pid];
        last = a.n_contrib[pid];
        C0 = rs.x; C1 = rs.y; C2 = rs.z; thr = rs.w;
    }
    const uint32_t cbase = a.ranges1[tile].y - a.ranges1[tile].x;
    // fused sort (no standalone phase-2 sort launches): wave 0 sorts a list of up to DS_WAVE_MAX2 into s_ids (and
    // back to s_e for the backward), the block sorts a longer one in place through the global scratch -- the same
    // two routines, so the same order, as k_tile_dsort / k_tile_dsort_long
    bool lds_ids = false;
#ifdef DG_DIAG_FWD2_NOSORT  // timing diagnostic only (wrong order)
    if (false) {
#else
    if (a.fuse_sort && n > 1) {
#endif
        uint32_t* scr = reinterpret_cast<uint32_t*>(s_sb);
        if (n <= DS_WAVE_MAX2) {
            if (w == 0) wave_sort_tile<DS_ROWS2>(a.ds, tile, lane, scr, scr + 256, scr + 256 + DS_WAVE_MAX2, s_ids, 1);
            lds_ids = true;
        } else {
            block_sort_long(a.ds, tile, scr, reinterpret_cast<uint32_t(*)[BS_RADIX]>(scr + BS_RADIX),
                            reinterpret_cast<uint32_t(*)[BS_WAVES]>(scr + BS_RADIX * (1 + BS_WAVES)),
                            reinterpret_cast<int*>(scr + BS_RADIX * (1 + BS_WAVES) + 2 * BS_WAVES));
        }
        __syncthreads();
    }
    for (int base = 0; base < n; base += FWD2_CHUNK) {
        const int cnt = n - base < FWD2_CHUNK ? n - base : FWD2_CHUNK;
        // the previous chunk is consumed by every wave; stop when every pixel of the tile has saturated
        if (!__syncthreads_or(thr < 1.0f ? 1 : 0)) break;
        for (int j = threadIdx.x; j < cnt + 4; j += 256) {
            float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;  // past the end: the null splat (opacity 0)
            if (j < cnt) {
                const uint32_t e = min(lds_ids ? s_ids[base + j] : a.s_e[rg.x + base + j], a.K - 1);
                const uint32_t g = min(a.eg[e], a.P - 1);
                const float4 s0 = a.sp[2 * g], s1 = a.sp[2 * g + 1];
                const float4 q = a.rgbi[g];
                const SplatExp k = splat_exp_coeffs(s0.z, s0.w, s1.x);
                r0 = make_float4(s0.x, s0.y, k.A, k.B);
                r1 = make_float4(k.C, s1.y, q.x, q.y);
                r2 = make_float4(q.z, q.w, __uint_as_float(g), 0.0f);
            }
            s_sb[j * 3 + 0] = r0; s_sb[j * 3 + 1] = r1; s_sb[j * 3 + 2] = r2;
        }
        __syncthreads();
#ifdef DG_DIAG_FWD2_NOCOMP  // timing diagnostic only (no compositing)
        if (cnt > 0) continue;
#endif
        for (int j0 = 0; j0 < cnt; j0 += 4) {
            if (!__any(thr < 1.0f)) break;  // every pixel of the wave saturated (or outside)
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int jj = j0 + u;
                const float4 Sa = s_sb[jj * 3 + 0], Sb = s_sb[jj * 3 + 1], Sc = s_sb[jj * 3 + 2];
                const float dy = Sa.y - pyf;
                const float bdy = Sa.w * dy, cdy2 = (Sb.x * dy) * dy;
                const float dx = Sa.x - pxf;
                const float p2 = fmaf(dx, fmaf(Sa.z, dx, bdy), cdy2);
                float al = Sb.y * __builtin_amdgcn_exp2f(p2);
                // forward.cu:451-475: skip power > 0 and alpha < 1/255, stop once T would fall below 1e-4
                const float ak = fminf(0.99f, al);
                const bool acc = !(p2 > 0.0f || ak < thr);
                al = acc ? ak : 0.0f;
                const float test_T = T * (1.0f - al);
                const bool term = test_T < 0.0001f;
                thr = term ? 2.0f : thr;
                al = term ? 0.0f : al;
                const float Tn = term ? T : test_T;
                last = (acc && !term) ? cbase + (uint32_t)(base + jj + 1) : last;
                if (COUNT) {  // LightGaussian count mode: pixels the splat contributes to (old forward.cu:481-487)
                    const uint32_t c = (uint32_t)__popcll(__ballot(acc && al != 0.0f));
                    if (c && lane == 0) atomicAdd(a.gcount + __float_as_uint(Sc.z), c);
                }
                const float wt = al * T;
                C0 = fmaf(Sb.z, wt, C0);
                C1 = fmaf(Sb.w, wt, C1);
                C2 = fmaf(Sc.x, wt, C2);
                D = fmaf(Sc.y, wt, D);
                T = Tn;
            }
        }
    }
    uint32_t mx = 0;
    if (inside) {
        const size_t HW = (size_t)a.W * a.H;
        a.final_T[pid] = T;
        a.n_contrib[pid] = last;
        const float o0 = fmaf(T, a.bg[0], C0);
        const float o1 = fmaf(T, a.bg[1], C1);
        const float o2 = fmaf(T, a.bg[2], C2);
        a.out_color[pid] = o0; a.out_color[HW + pid] = o1; a.out_color[2 * HW + pid] = o2;
        a.img_color[pid] = o0; a.img_color[HW + pid] = o1; a.img_color[2 * HW + pid] = o2;
        a.out_invd[pid] = D;
        a.img_invd[pid] = D;
        mx = last;
    }
    mx = wave_max_u32(mx);
    if (lane == 0) s_mx[w] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t m01 = s_mx[0] > s_mx[1] ? s_mx[0] : s_mx[1], m23 = s_mx[2] > s_mx[3] ? s_mx[2] : s_mx[3];
        a.max_contrib[tile] = m01 > m23 ? m01 : m23;
    }
}

// Phase 2 with the alphas and the compositing chain split (DG_FWD2_SPLIT; k_render_fwd2's arithmetic, bit for bit).
// k_render_fwd2 runs nearly alone on the chip with one wave per SIMD, so its time is one wave's instruction stream
// per splat.  Here a 1024-thread block per tile: all 16 waves compute the alphas of a sub-chunk of F2X_SUB splats
// for the tile's 256 pixels (4 pixels per splat-lane team, 16 waves sharing the SIMDs) into LDS, then the four
// pixel waves run only the transmittance / colour chain over them.  The stored value is min(0.99, o exp2(power)), or
// -1 when power > 0 (then `ak < thr` rejects it exactly as `power > 0 ||` does).
#ifndef DG_FWD2X_CHUNK
#define DG_FWD2X_CHUNK 512
#endif
#ifndef DG_FWD2X_SUB
#define DG_FWD2X_SUB 32
#endif
constexpr int F2X_CHUNK = DG_FWD2X_CHUNK, F2X_SUB = DG_FWD2X_SUB;
template <bool COUNT>
__global__ void __launch_bounds__(1024) k_render_fwd2x(RenderArgs a) {
    __shared__ __attribute__((aligned(16))) float4 s_sb[(F2X_CHUNK + 4) * 3];  // (also the sort's scratch)
    __shared__ float s_al[F2X_SUB * 256];
    __shared__ uint32_t s_mx[4];
    __shared__ uint32_t s_ids[DS_WAVE_MAX2];
    static_assert((F2X_CHUNK + 4) * 12 >= BS_RADIX * (1 + BS_WAVES) + 2 * BS_WAVES + 1, "sort scratch");
    static_assert(F2X_CHUNK % F2X_SUB == 0 && F2X_SUB % 4 == 0, "sub-chunks");
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const bool pix = t < 256;  // the four pixel waves (k_render_fwd2's mapping)
    const int tile = blockIdx.x;
    if (a.probe && blockIdx.x == 0 && threadIdx.x == 0) a.probe[1] = a.counters[CNT_K2];
    if (tile >= a.num_tiles || !a.unfinished[tile]) return;  // block-uniform: finished in phase 1
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int p = t & 255;                                  // pixel of this thread in the alpha pass (= t for pix)
    const int px = tx * GS_TILE_X + (p & 15), py = ty * GS_TILE_Y + (p >> 4);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;
    float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f, D = 0.0f, thr = 2.0f;
    uint32_t last = 0;
    const size_t pid = inside ? (size_t)py * a.W + px : 0;
    if (pix && inside) {
        const float4 rs = a.resume[pid];
        T = a.final_T[pid];
        D = a.img_invd[pid];
        last = a.n_contrib[pid];
        C0 = rs.x; C1 = rs.y; C2 = rs.z; thr = rs.w;
    }
    const uint32_t cbase = a.ranges1[tile].y - a.ranges1[tile].x;
    const uint2 rg = a.ranges[tile];
    const int n = (int)(rg.y - rg.x);
    bool lds_ids = false;
    if (a.fuse_sort && n > 1) {
        uint32_t* scr = reinterpret_cast<uint32_t*>(s_sb);
        if (n <= DS_WAVE_MAX2) {
            if (w == 0) wave_sort_tile<DS_ROWS2>(a.ds, tile, lane, scr, scr + 256, scr + 256 + DS_WAVE_MAX2, s_ids, 1);
            lds_ids = true;
        } else {
            block_sort_long(a.ds, tile, scr, reinterpret_cast<uint32_t(*)[BS_RADIX]>(scr + BS_RADIX),
                            reinterpret_cast<uint32_t(*)[BS_WAVES]>(scr + BS_RADIX * (1 + BS_WAVES)),
                            reinterpret_cast<int*>(scr + BS_RADIX * (1 + BS_WAVES) + 2 * BS_WAVES));
        }
        __syncthreads();
    }
    const int team = t >> 8;  // alpha pass: splat lanes team, team + 4, ...
    for (int base = 0; base < n; base += F2X_CHUNK) {
        const int cnt = n - base < F2X_CHUNK ? n - base : F2X_CHUNK;
        if (!__syncthreads_or((pix && thr < 1.0f) ? 1 : 0)) break;
        for (int j = t; j < cnt + 4; j += 1024) {
            float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;
            if (j < cnt) {
                const uint32_t e = min(lds_ids ? s_ids[base + j] : a.s_e[rg.x + base + j], a.K - 1);
                const uint32_t g = min(a.eg[e], a.P - 1);
                const float4 s0 = a.sp[2 * g], s1 = a.sp[2 * g + 1];
                const float4 q = a.rgbi[g];
                const SplatExp k = splat_exp_coeffs(s0.z, s0.w, s1.x);
                r0 = make_float4(s0.x, s0.y, k.A, k.B);
                r1 = make_float4(k.C, s1.y, q.x, q.y);
                r2 = make_float4(q.z, q.w, __uint_as_float(g), 0.0f);
            }
            s_sb[j * 3 + 0] = r0; s_sb[j * 3 + 1] = r1; s_sb[j * 3 + 2] = r2;
        }
        __syncthreads();
        for (int sub = 0; sub < cnt; sub += F2X_SUB) {
            if (!__syncthreads_or((pix && thr < 1.0f) ? 1 : 0)) break;  // (also: the last chain is done with s_al)
#pragma unroll 4
            for (int jj = team; jj < F2X_SUB; jj += 4) {
                const int j = sub + jj;
                float v = -1.0f;
                if (j < cnt) {
                    const float4 Sa = s_sb[j * 3 + 0], Sb = s_sb[j * 3 + 1];
                    const float dy = Sa.y - pyf;
                    const float bdy = Sa.w * dy, cdy2 = (Sb.x * dy) * dy;
                    const float dx = Sa.x - pxf;
                    const float p2 = fmaf(dx, fmaf(Sa.z, dx, bdy), cdy2);
                    const float ak = fminf(0.99f, Sb.y * __builtin_amdgcn_exp2f(p2));
                    v = p2 > 0.0f ? -1.0f : ak;
                }
                s_al[jj * 256 + p] = v;
            }
            __syncthreads();
            if (pix) {
                const int m = cnt - sub < F2X_SUB ? cnt - sub : F2X_SUB;
                for (int j0 = 0; j0 < m; j0 += 4) {
                    if (!__any(thr < 1.0f)) break;
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int jj = j0 + u;
                        if (jj >= m) break;  // wave-uniform
                        const int j = sub + jj;
                        const float4 Sb = s_sb[j * 3 + 1], Sc = s_sb[j * 3 + 2];
                        const float ak = s_al[jj * 256 + p];
                        const bool acc = !(ak < thr);
                        float al = acc ? ak : 0.0f;
                        const float test_T = T * (1.0f - al);
                        const bool term = test_T < 0.0001f;
                        thr = term ? 2.0f : thr;
                        al = term ? 0.0f : al;
                        const float Tn = term ? T : test_T;
                        last = (acc && !term) ? cbase + (uint32_t)(base + j + 1) : last;
                        if (COUNT) {
                            const uint32_t c = (uint32_t)__popcll(__ballot(acc && al != 0.0f));
                            if (c && lane == 0) atomicAdd(a.gcount + __float_as_uint(Sc.z), c);
                        }
                        const float wt = al * T;
                        C0 = fmaf(Sb.z, wt, C0);
                        C1 = fmaf(Sb.w, wt, C1);
                        C2 = fmaf(Sc.x, wt, C2);
                        D = fmaf(Sc.y, wt, D);
                        T = Tn;
                    }
                }
            }
        }
        __syncthreads();  // the next chunk's gather overwrites s_sb
    }
    uint32_t mx = 0;
    if (pix && inside) {
        const size_t HW = (size_t)a.W * a.H;
        a.final_T[pid] = T;
        a.n_contrib[pid] = last;
        const float o0 = fmaf(T, a.bg[0], C0);
        const float o1 = fmaf(T, a.bg[1], C1);
        const float o2 = fmaf(T, a.bg[2], C2);
        a.out_color[pid] = o0; a.out_color[HW + pid] = o1; a.out_color[2 * HW + pid] = o2;
        a.img_color[pid] = o0; a.img_color[HW + pid] = o1; a.img_color[2 * HW + pid] = o2;
        a.out_invd[pid] = D;
        a.img_invd[pid] = D;
        mx = last;
    }
    mx = wave_max_u32(mx);
    if (pix && lane == 0) s_mx[w] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t m01 = s_mx[0] > s_mx[1] ? s_mx[0] : s_mx[1], m23 = s_mx[2] > s_mx[3] ? s_mx[2] : s_mx[3];
        a.max_contrib[tile] = m01 > m23 ? m01 : m23;
    }
}

// the precise cull's threshold per opacity, exactly as the binning evaluates it (parity probe of gs_crlogf)
__global__ void __launch_bounds__(256) k_cull_log_threshold(int64_t n, const float* __restrict__ opacity,
                                                            float* __restrict__ thr) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) thr[i] = gs_crlogf(opacity[i] / (1.0f / 255.0f));
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
    // both sources land in registers (a pointer to either would put the local copy on the stack)
    float cbuf[6];
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) cbuf[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        const f3 s = {a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]};
        const f4 q = {a.rotations[4 * idx], a.rotations[4 * idx + 1], a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]};
        cov3d_fwd(s, a.scale_mod, q, cbuf);
    }
    const float* cov3D = cbuf;
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
    if (a.P > 0) k_preprocess<<<preprocess_blocks(a.P), 256, 0, s>>>(a);
}
uint32_t preprocess_blocks(int P) { return (uint32_t)((P + 256 * PRE_PT - 1) / (256 * PRE_PT)); }
void launch_depth_hist(int P, const uint32_t* dkey, const uint32_t* cnt, uint32_t* hist, hipStream_t s) {
    const int per = DH_THREADS * DH_ITEMS;
    if (P > 0) k_depth_hist<<<(P + per - 1) / per, DH_THREADS, 0, s>>>(P, dkey, cnt, hist);
}
void launch_depth_hist_cut(int P, const uint32_t* dkey, const uint32_t* cnt, uint32_t* hist, uint32_t cap,
                           uint32_t* counters, uint32_t* tile_cnt, uint32_t* tile_cnt2, uint32_t num_tiles,
                           const unsigned long long* rect_part, uint32_t nparts, uint32_t* probe, hipStream_t s) {
    // (one launch -- every block flushing, a ticket, the last block cutting -- measured 72 us against 8 + 7 here)
    launch_depth_hist(P, dkey, cnt, hist, s);
    launch_depth_cut(hist, cap, counters, tile_cnt, tile_cnt2, num_tiles, rect_part, nparts, probe, s);
}
void launch_depth_cut(const uint32_t* hist, uint32_t cap, uint32_t* counters, uint32_t* tile_cnt, uint32_t* tile_cnt2,
                      uint32_t num_tiles, const unsigned long long* rect_part, uint32_t nparts, uint32_t* probe,
                      hipStream_t s) {
    k_depth_cut<<<1, 1024, 0, s>>>(hist, cap, counters, tile_cnt, tile_cnt2, num_tiles, rect_part, nparts, probe);
}
void launch_bin(int phase, const BinArgs& a, uint32_t* total, void* scan_tmp, hipStream_t s, hipEvent_t wait_before_emit) {
    if (a.P <= 0) return;
    const bool fat = phase == 1 ? DG_BIN_FAT1 > 1 : DG_BIN_FAT2 > 1;
    const int span = fat ? (phase == 1 ? fat_span<1>() : fat_span<2>()) : EMIT_RANKS;
    const int waves = (a.P + span - 1) / span;
    const int blocks = (waves + 3) / 4;
    const uint32_t* gate = phase == 2 ? a.counters + CNT_UNFINISHED : nullptr;
    if (fat) {
        if (phase == 2) k_bin_count_fat<2><<<blocks, 256, 0, s>>>(a);
        else k_bin_count_fat<1><<<blocks, 256, 0, s>>>(a);
    } else if (phase == 2) k_bin_count<2><<<blocks, 256, 0, s>>>(a);
    else k_bin_count<1><<<blocks, 256, 0, s>>>(a);
    if ((uint32_t)waves <= BIN_OFFSETS_MAX_N) {  // one launch: wave offsets + tile ranges, tile_cnt -> range starts (cursors)
        bin_offsets(a.wtot, (uint32_t)waves, total, a.tile_cnt, (uint32_t)a.num_tiles, a.ranges, s, gate,
                    a.colors_later != 0);
    } else {
        exclusive_scan(a.wtot, (uint32_t)waves, a.wtot, total, scan_tmp, s, gate);
        tile_offsets(a.tile_cnt, (uint32_t)a.num_tiles, a.ranges, s, gate);
    }
    if (wait_before_emit) (void)hipStreamWaitEvent(s, wait_before_emit, 0);  // the emission reads the SH rows
    if (fat) {
        if (phase == 2) k_bin_emit_fat<2><<<blocks, 256, 0, s>>>(a);
        else k_bin_emit_fat<1><<<blocks, 256, 0, s>>>(a);
    } else if (phase == 2) {
        k_bin_emit<2><<<blocks + (a.ohist ? order_blocks(a.num_tiles) : 0) + (a.unf_sorted ? 1 : 0), 256, 0, s>>>(a);
    }
    else k_bin_emit<1><<<blocks, 256, 0, s>>>(a);
}
void launch_binned_colors(const BinArgs& a, hipStream_t s) {
    if (a.P > 0) k_binned_colors<<<(a.P + 255) / 256, 256, 0, s>>>(a);
}
size_t bin_scan_temp_bytes(int P) { return scan_temp_bytes((uint32_t)((P + EMIT_RANKS - 1) / EMIT_RANKS)); }
int bin_waves(int P) { return (P + EMIT_RANKS - 1) / EMIT_RANKS; }
void launch_unfinished_sat(const uint32_t* counters, const uint8_t* unfinished, int tiles_x, int tiles_y,
                           uint32_t* sat, hipStream_t s, uint32_t* probe) {
    k_sat_rows<<<(tiles_y + 1 + 3) / 4, 256, 0, s>>>(counters, unfinished, tiles_x, tiles_y, sat, probe);
    k_sat_cols<<<(tiles_x + 3) / 4, 256, 0, s>>>(counters, tiles_x, tiles_y, sat);
}
bool bin_emit_orders() { return !(DG_BIN_FAT2 > 1); }  // k_bin_emit<2> runs order_hist_piece (BinArgs::ohist)
bool render_fwd2_orders() {  // the phase-2 launch writes RenderArgs::order (the backward skips k_bwd_order)
#if defined(DG_PHASE2_WAVE_PER_TILE) || defined(DG_FWD2_SPLIT)
    return false;
#else
    return true;
#endif
}
void launch_render_fwd(const RenderArgs& a, hipStream_t s) {
    if (a.num_tiles <= 0) return;
    const int blocks = (a.num_tiles + 3) / 4;
#ifndef DG_PHASE2_WAVE_PER_TILE  // A/B switch: phase 2 with k_render_fwd's one wave per tile
    if (a.phase == 2) {
#ifdef DG_FWD2_SPLIT
        if (a.gcount) k_render_fwd2x<true><<<a.num_tiles, 1024, 0, s>>>(a);
        else k_render_fwd2x<false><<<a.num_tiles, 1024, 0, s>>>(a);
#else
        const int g2 = (a.unf_list ? (a.num_tiles < FWD2_GRID ? a.num_tiles : FWD2_GRID) : a.num_tiles) +
                       (a.order ? (a.ohist ? order_blocks(a.num_tiles) : 1) : 0);
        if (a.gcount) k_render_fwd2<true><<<g2, 256, 0, s>>>(a);
        else k_render_fwd2<false><<<g2, 256, 0, s>>>(a);
#endif
        return;
    }
#endif
    if (a.gcount) {
        if (a.phase == 2) k_render_fwd<2, true><<<blocks, 256, 0, s>>>(a);
        else k_render_fwd<1, true><<<blocks, 256, 0, s>>>(a);
    } else {
        if (a.phase == 2) k_render_fwd<2, false><<<blocks, 256, 0, s>>>(a);
        else k_render_fwd<1, false><<<blocks, 256, 0, s>>>(a);
    }
}

// important_score = opacity x contributing pixels: the reference adds the opacity once per contributing pixel
// (old forward.cu:486); here the count is exact (integer atomics) and the product is formed once.
__global__ void __launch_bounds__(256) k_count_score(int P, const int* __restrict__ radii,
                                                     const float4* __restrict__ sp, const uint32_t* __restrict__ gcount,
                                                     float* __restrict__ score) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint32_t n = gcount[i];
    score[i] = (radii[i] > 0 && n) ? (float)n * sp[2 * i + 1].y : 0.0f;
}
void launch_count_score(int P, const int* radii, const float4* sp, const uint32_t* gcount, float* score,
                        hipStream_t s) {
    if (P > 0) k_count_score<<<(P + 255) / 256, 256, 0, s>>>(P, radii, sp, gcount, score);
}
void launch_cull_log_threshold(int64_t n, const float* opacity, float* thr, hipStream_t s) {
    if (n > 0) k_cull_log_threshold<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(n, opacity, thr);
}
void launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t s) {
    if (P > 0) k_mark_visible<<<(P + 255) / 256, 256, 0, s>>>(P, means3D, view, present);
}
void launch_filter(const PreArgs& a, hipStream_t s) {
    if (a.P > 0) k_filter<<<(a.P + 255) / 256, 256, 0, s>>>(a);
}

}  // namespace gs

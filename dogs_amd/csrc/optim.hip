// optim.hip -- optimizer-side kernels of a training view (optim.h).
//
// k_adam_multi      SparseGaussianAdam.step (diff_gaussian_rasterization/__init__.py:303-332 -> adam.cu:10-38) for
//                   every parameter group in one launch (optionally with the ADMM proximal gradient of a block
//                   trainer, slave_gaussian_trainer.py:161-202, added to the visible rows' gradient), plus the view's
//                   densification statistics
//                   (gaussian_trainer.py:433-438 max_radii2D, gaussian_splat_model.py:533-541 add_densification_stats).
//                   Blocks are assigned to groups in contiguous ranges (block-uniform group, scalar kernel-argument
//                   loads); each lane updates 4 consecutive floats (float4 when the group is 16-byte aligned).
//                   HBM-bound: 28 B per visible float (read param/grad/m/v, write param/m/v).
// k_densify_*       densify_and_prune (gaussian_splat_model.py:434-531) as stream compaction: clone/split selection,
//                   keep flags over the candidate rows [originals not split | clones | split children], one gather.
#include <hip/hip_runtime.h>
#include <math.h>

#include "optim.h"

namespace gs {

namespace {

__device__ __forceinline__ float adam_one(float p, float gr, float& m, float& v, float lr, float b1, float b2, float eps) {
    // adam.cu:21-28 (same expression shape as aux_kernels.hip k_adam)
    const float em = fmaf(b1, m, (1.0f - b1) * gr);
    const float ev = fmaf(b2, v, ((1.0f - b2) * gr) * gr);
    m = em;
    v = ev;
    return p + (-lr * em / (sqrtf(ev) + eps));
}

typedef float nt_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load4(const float* p) {
    const nt_f4 x = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void nt_store4(float* p, float4 v) {
    const nt_f4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<nt_f4*>(p));
}

#ifndef DG_ADAM_CHUNKS
#define DG_ADAM_CHUNKS 1
#endif
constexpr int ADAM_CHUNKS = DG_ADAM_CHUNKS;  // float4 chunks per lane

// Backward of the parameter activations (gaussian_splat_model.py get_opacity / get_scaling / get_quaternion), shared
// by k_activate_bwd and the activation-folded Adam so both routes evaluate the same expressions.
// (g (1 - y)) y: torch's sigmoid_backward association, so the native step's opacity gradient equals the autograd route's
__device__ __forceinline__ float sigmoid_bwd(float g, float v) { return (g * (1.0f - v)) * v; }
// exp's backward of scaling column r, with the scale regulariser lambda_scale mean(prod(scaling, 1))
// (gaussian_trainer.py:407-408): its gradient reg prod / s_r joins the rasterizer's before exp's backward.  torch's
// prod backward is result / input when the input holds no zero and the product of the other columns otherwise
// (prod_safe_zeros_backward), for every row of the tensor as soon as one scaling is 0 (torch tests the whole input).
// zmode 1: some scaling of the step is 0 (the activation pass's stamp), 0: none; -1: decide per row (the C-ABI
// activation backward, which has no stamp).  An underflowed scale (exp of a raw value below ~-87) so gives a finite
// gradient instead of 0/0, and the rows without a zero round as torch rounds them.
__device__ __forceinline__ float exp_bwd(float g, const float* __restrict__ s3, int r, float reg, int zmode) {
    if (reg != 0.0f) {
        float d;
        if (zmode > 0 || (zmode < 0 && (s3[0] == 0.0f || s3[1] == 0.0f || s3[2] == 0.0f)))
            d = r == 0 ? s3[2] * s3[1] : r == 1 ? s3[0] * s3[2] : s3[0] * s3[1];
        else
            d = ((s3[0] * s3[2]) * s3[1]) / s3[r];  // torch.prod's row order on the GPU (k_row_prod_fwd)
        return (g + reg * d) * s3[r];
    }
    return g * s3[r];
}
// F.normalize(x, eps 1e-12): d(x / n) = g / n - y (y . g) / n, or g / eps on the clamped denominator.  The norm is
// summed pairwise, (x0^2 + x1^2) + (x2^2 + x3^2), as torch's vector_norm does (tools/act_match_probe.py: the forward
// then equals F.normalize bit for bit; sigmoid and exp already do)
__device__ __forceinline__ float4 normalize_bwd(float4 x, float4 g) {
    const float n = sqrtf((x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w));
    if (n >= 1e-12f) {
        // torch's autograd of x / n.clamp_min(eps).expand_as(x), op for op (tools/normalize_bwd_probe.py: bit-identical
        // on 4M elements): div's other-gradient -g (y / n), its expand summed pairwise, then g / n + s y
        const float4 y = make_float4(x.x / n, x.y / n, x.z / n, x.w / n);
        const float s = (-g.x * (y.x / n) + -g.y * (y.y / n)) + (-g.z * (y.z / n) + -g.w * (y.w / n));
        return make_float4(g.x / n + s * y.x, g.y / n + s * y.y, g.z / n + s * y.z, g.w / n + s * y.w);
    }
    return make_float4(g.x / 1e-12f, g.y / 1e-12f, g.z / 1e-12f, g.w / 1e-12f);
}

__device__ __forceinline__ float f4get(const float4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(float4& v, int j, float x) {
    if (j == 0) v.x = x; else if (j == 1) v.y = x; else if (j == 2) v.z = x; else v.w = x;
}

// one 256-thread work block (group chunks, or the row blocks past start[n])
__device__ __forceinline__ void adam_block(const AdamMultiArgs& a, const uint32_t blk) {
    if (blk >= a.start[a.n]) {  // row blocks: the status snapshot and the densification statistics, a row per lane
        const uint32_t i = (blk - a.start[a.n]) * 256u + threadIdx.x;
        if (i >= a.N) return;
        const bool vis = a.visible ? a.visible[i] != 0 : a.vis_radii[i] > 0;
        if (a.status_out) a.status_out[i] = (uint8_t)((vis ? 1u : 0u) | (!a.hot || a.hot[i] != 0u ? 2u : 0u));
        if (!a.radii || !vis) return;
        // max_radii2D[vis] = max(max_radii2D[vis], radii[vis]) (float result: radii promote to float)
        const float r = (float)a.radii[i];
        const float mr = a.max_radii2D[i];
        a.max_radii2D[i] = r > mr ? r : mr;
        // xyz_gradient_accum[vis] += ||grad[vis, :2]||, denom[vis] += 1 (a row no tile binned has none)
        float gx = 0.0f, gy = 0.0f;
        if (!a.hot || a.hot[i] != 0u) {
            gx = a.dmeans2D[(size_t)i * a.dm_stride];
            gy = a.dmeans2D[(size_t)i * a.dm_stride + 1];
            if (a.depth_thr > 0.0f) {  // torch.minimum(ones, (depth / thr) ** 2), then grad * factor
                // torch divides by a Python scalar as a multiply by its float reciprocal (div_true_kernel_cuda)
                const float q = a.depth[i] * (1.0f / a.depth_thr);
                const float sq = q * q;
                const float f = (sq < 1.0f || sq != sq) ? sq : 1.0f;  // torch.minimum propagates NaN
                gx = gx * f;
                gy = gy * f;
            }
        }
        a.grad_accum[i] += sqrtf(gx * gx + gy * gy);
        a.denom[i] += 1.0f;
        return;
    }
    int k = 0;
    while (k + 1 < a.n && blk >= a.start[k + 1]) k++;  // block-uniform
    const AdamGroup g = a.g[k];
    // N * M < 2^32 (checked on the host): 32-bit index math, one division per lane.  Each lane owns ADAM_CHUNKS
    // float4 chunks, 256 * 4 floats apart (coalesced per chunk), all loads issued before any update.
    const uint32_t total = a.N * g.M;
    const float b1 = a.b1, b2 = a.b2;
    const uint32_t base = 4u * ((blk - a.start[k]) * 256u * ADAM_CHUNKS + threadIdx.x);
    float4 p[ADAM_CHUNKS], gr[ADAM_CHUNKS], m[ADAM_CHUNKS], v[ADAM_CHUNKS];
    bool vis[ADAM_CHUNKS][4], act[ADAM_CHUNKS], full[ADAM_CHUNKS];
#pragma unroll
    for (int c = 0; c < ADAM_CHUNKS; c++) {
        const uint32_t e0 = base + 1024u * c;
        act[c] = false;
        full[c] = false;
        if (e0 >= total) continue;
        const uint32_t gi0 = e0 / g.M, r0 = e0 - gi0 * g.M;
        uint32_t gi = gi0, r = r0;
        bool hot = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool in = e0 + j < total;
            if (a.status) {
                const uint32_t st = in ? a.status[gi] : 0u;
                vis[c][j] = (st & 1u) != 0u;
                hot |= (st & 2u) != 0u;
            } else {
                vis[c][j] = in && (a.visible ? a.visible[gi] != 0 : a.vis_radii[gi] > 0);
                if (a.hot && in) hot |= a.hot[gi] != 0u;
            }
            act[c] |= vis[c][j];
            if (++r == g.M) { r = 0; gi++; }
        }
        if (!act[c]) continue;
        // no binned row in the chunk: its rasterizer gradient is zero
        const bool zero_grad = a.status ? !hot : (a.hot && !hot);
        full[c] = g.vec && e0 + 4 <= total;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (full[c]) {
#ifndef DG_ADAM_CACHED
            p[c] = nt_load4(g.param + e0);
            gr[c] = zero_grad ? z4 : nt_load4(g.grad + e0);
            m[c] = nt_load4(g.m + e0); v[c] = nt_load4(g.v + e0);
#else
            p[c] = *reinterpret_cast<const float4*>(g.param + e0);
            gr[c] = zero_grad ? z4 : *reinterpret_cast<const float4*>(g.grad + e0);
            m[c] = *reinterpret_cast<const float4*>(g.m + e0);
            v[c] = *reinterpret_cast<const float4*>(g.v + e0);
#endif
        } else {
            p[c] = gr[c] = m[c] = v[c] = z4;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (e0 + j >= total) continue;
                f4set(p[c], j, g.param[e0 + j]);
                f4set(m[c], j, g.m[e0 + j]);
                f4set(v[c], j, g.v[e0 + j]);
                if (!zero_grad) f4set(gr[c], j, g.grad[e0 + j]);
            }
        }
        // the activation's backward (dL/d activated -> dL/d raw), before the proximal term and the moments
        if (g.gmode == 1) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (e0 + j < total) f4set(gr[c], j, sigmoid_bwd(f4get(gr[c], j), g.act[gi0 + j]));
        } else if (g.gmode == 2) {
            uint32_t gj = gi0, rj = r0;
            const int zmode = g.zero_stamp ? (*g.zero_stamp == g.stamp ? 1 : 0) : -1;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (e0 + j < total)
                    f4set(gr[c], j, exp_bwd(f4get(gr[c], j), g.act + 3 * (size_t)gj, (int)rj, g.reg, zmode));
                if (++rj == 3u) { rj = 0; gj++; }
            }
        } else if (g.gmode == 3) {
            gr[c] = normalize_bwd(p[c], gr[c]);  // M = 4: the chunk is the row
        }
        if (g.u) {  // the ADMM proximal gradient joins the loss gradient before the moments see it
            float4 u, z;
            if (full[c]) {
                u = nt_load4(g.u + e0); z = nt_load4(g.z + e0);
            } else {
                u = z = z4;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (e0 + j < total) { f4set(u, j, g.u[e0 + j]); f4set(z, j, g.z[e0 + j]); }
            }
            gr[c].x += g.coef * ((p[c].x + u.x) - z.x); gr[c].y += g.coef * ((p[c].y + u.y) - z.y);
            gr[c].z += g.coef * ((p[c].z + u.z) - z.z); gr[c].w += g.coef * ((p[c].w + u.w) - z.w);
        }
    }
#pragma unroll
    for (int c = 0; c < ADAM_CHUNKS; c++) {
        const uint32_t e0 = base + 1024u * c;
        if (!act[c]) continue;
        if (vis[c][0]) p[c].x = adam_one(p[c].x, gr[c].x, m[c].x, v[c].x, g.lr, b1, b2, g.eps);
        if (vis[c][1]) p[c].y = adam_one(p[c].y, gr[c].y, m[c].y, v[c].y, g.lr, b1, b2, g.eps);
        if (vis[c][2]) p[c].z = adam_one(p[c].z, gr[c].z, m[c].z, v[c].z, g.lr, b1, b2, g.eps);
        if (vis[c][3]) p[c].w = adam_one(p[c].w, gr[c].w, m[c].w, v[c].w, g.lr, b1, b2, g.eps);
        if (full[c]) {
#ifndef DG_ADAM_CACHED  // streaming (non-temporal) loads and stores: every byte is touched once (327 -> 269 us)
            nt_store4(g.param + e0, p[c]); nt_store4(g.m + e0, m[c]); nt_store4(g.v + e0, v[c]);
#else
            *reinterpret_cast<float4*>(g.param + e0) = p[c];
            *reinterpret_cast<float4*>(g.m + e0) = m[c];
            *reinterpret_cast<float4*>(g.v + e0) = v[c];
#endif
            continue;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (!vis[c][j]) continue;
            g.param[e0 + j] = f4get(p[c], j);
            g.m[e0 + j] = f4get(m[c], j);
            g.v[e0 + j] = f4get(v[c], j);
        }
    }
}

// A full grid (one work block per block), or -- grid_cap, the native step's overlapped SH update -- a capped grid that
// strides over the work blocks, leaving compute units to the stream it overlaps (a full-grid update filled every CU
// and held the next forward's one-block depth cut back ~150 us).
__global__ void __launch_bounds__(256) k_adam_multi(AdamMultiArgs a) {
    for (uint32_t blk = blockIdx.x; blk < a.nblocks; blk += gridDim.x) adam_block(a, blk);
}


// ---- densify_and_prune

__device__ __forceinline__ float max_scale(const float* s) {
    // torch.max(get_scaling, dim=1).values, get_scaling = exp(_scaling)
    const float a = expf(s[0]), b = expf(s[1]), c = expf(s[2]);
    const float ab = a > b ? a : b;
    return ab > c ? ab : c;
}

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

// densify_and_clone / densify_and_split selection (gaussian_splat_model.py:434-441, 464-469):
// grads = accum / denom (NaN -> 0); clone: |grads| >= thr and max scale <= percent_dense * extent;
// split: grads >= thr and max scale > percent_dense * extent (clones are appended with padded grad 0: never split).
__global__ void __launch_bounds__(256) k_densify_select(DensifyArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.N) return;
    float g = a.grad_accum[i] / a.denom[i];
    if (g != g) g = 0.0f;
    const float ms = max_scale(a.scaling + 3 * (size_t)i);
    a.clone_flag[i] = (fabsf(g) >= a.grad_threshold && ms <= a.dense_extent) ? 1u : 0u;
    a.split_flag[i] = (g >= a.grad_threshold && ms > a.dense_extent) ? 1u : 0u;
}

__global__ void __launch_bounds__(256) k_densify_lists(DensifyArgs a, const uint32_t* __restrict__ clone_pos,
                                                       const uint32_t* __restrict__ split_pos,
                                                       uint32_t* __restrict__ clone_idx, uint32_t* __restrict__ split_idx) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.N) return;
    if (a.clone_flag[i]) clone_idx[clone_pos[i]] = i;
    if (a.split_flag[i]) split_idx[split_pos[i]] = i;
}

// Candidate row r: r < N original r (dropped when split), then nc clones, then replicas x ns split children
// (torch .repeat(replicas, 1): replica-major).  src = the original it comes from; child = replica index + 1 or 0.
struct Cand { uint32_t src; int kind; };  // kind 0 original, 1 clone, 2 child
__device__ __forceinline__ Cand cand_of(const RebuildArgs& a, uint32_t r) {
    if (r < a.d.N) return {r, 0};
    r -= a.d.N;
    if (r < a.nc) return {a.clone_idx[r], 1};
    r -= a.nc;
    return {a.split_idx[r % a.ns], 2};
}

// normalize_quaternion + quaternion_to_rotation_mat (utils.py:20-67), one op at a time as torch evaluates them;
// row c of R only (c may differ per lane: selects, no indexed local array)
__device__ __forceinline__ void rot_row(const float* q, int c, float& a0, float& a1, float& a2) {
    const float n = sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
    const float r = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
    if (c == 0) {
        a0 = 1.0f - 2.0f * (y * y + z * z); a1 = 2.0f * (x * y - r * z); a2 = 2.0f * (x * z + r * y);
    } else if (c == 1) {
        a0 = 2.0f * (x * y + r * z); a1 = 1.0f - 2.0f * (x * x + z * z); a2 = 2.0f * (y * z - r * x);
    } else {
        a0 = 2.0f * (x * z - r * y); a1 = 2.0f * (y * z + r * x); a2 = 1.0f - 2.0f * (x * x + y * y);
    }
}

// split child k (gaussian_splat_model.py:471-483): xyz = R(q) @ sample + xyz (bmm: k = 3 fma chain),
// scaling = log(exp(s) / (0.8 * replicas))
__device__ __forceinline__ float child_xyz(const RebuildArgs& a, uint32_t k, uint32_t src, int c) {
    float r0, r1, r2;
    rot_row(a.d.rot + 4 * (size_t)src, c, r0, r1, r2);
    const float* smp = a.samples + 3 * (size_t)k;
    const float dot = fmaf(r2, smp[2], fmaf(r1, smp[1], r0 * smp[0]));
    return dot + a.d.xyz[3 * (size_t)src + c];
}
__device__ __forceinline__ float child_scaling(const RebuildArgs& a, uint32_t src, int c) {
    // torch divides by a Python scalar on the GPU as a multiplication by its float reciprocal
    const float inv = 1.0f / (float)(0.8 * (double)a.replicas);
    return logf(expf(a.d.scaling[3 * (size_t)src + c]) * inv);
}

// prune mask (gaussian_splat_model.py:516-528) of a candidate row.  densification_postfix reset max_radii2D to zeros
// before this test, so big_points_vs reduces to 0 > max_screen_size, as in the reference.
__global__ void __launch_bounds__(256) k_densify_keep(RebuildArgs a) {
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;
    const uint32_t C = a.d.N + a.nc + a.replicas * a.ns;
    if (r >= C) return;
    const Cand c = cand_of(a, r);
    uint32_t keep = 1u;
    if (c.kind == 0 && a.d.split_flag[c.src]) keep = 0u;
    float z, s[3];
    if (c.kind == 2) {
        const uint32_t k = r - a.d.N - a.nc;
        z = child_xyz(a, k, c.src, 2);
        for (int j = 0; j < 3; j++) s[j] = child_scaling(a, c.src, j);
    } else {
        z = a.d.xyz[3 * (size_t)c.src + 2];
        for (int j = 0; j < 3; j++) s[j] = a.d.scaling[3 * (size_t)c.src + j];
    }
    bool prune = sigmoid_f(a.d.opacity[c.src]) < a.min_opacity;
    if (a.use_bbox) prune = prune || z < a.bbox_z;
    if (a.use_screen) prune = prune || (0.0f > a.max_screen) || max_scale(s) > a.big_extent;
    if (prune) keep = 0u;
    a.keep[r] = keep;
}

// One lane per (candidate, float) of one group; blocks are assigned to the six groups in contiguous ranges
// (gstart[q], block-uniform group), so every lane of a wave reads and writes one array, coalesced.  Params from the
// source row (children: new xyz / scaling), Adam moments copied for originals, zero for appended rows
// (cat_tensors_to_optimizer: zeros_like).
template <int Q>
__device__ __forceinline__ void gather_group(const RebuildArgs& a, const uint32_t* __restrict__ keep_pos, uint32_t t,
                                             uint32_t C) {
    const uint32_t w = a.d.width[Q];
    const uint32_t r = t / w;
    if (r >= C || !a.keep[r]) return;
    const uint32_t e = t - r * w;
    const Cand c = cand_of(a, r);
    const float* src = Q == 0 ? a.d.xyz : Q == 1 ? a.d.f_dc : Q == 2 ? a.d.f_rest : Q == 3 ? a.d.opacity
                     : Q == 4 ? a.d.scaling : a.d.rot;
    float val;
    if (Q == 0 && c.kind == 2) val = child_xyz(a, r - a.d.N - a.nc, c.src, (int)e);
    else if (Q == 4 && c.kind == 2) val = child_scaling(a, c.src, (int)e);
    else val = src[(size_t)c.src * w + e];
    const size_t o = (size_t)keep_pos[r] * w + e;
    a.out_p[Q][o] = val;
    if (a.out_m[Q]) a.out_m[Q][o] = (c.kind == 0 && a.d.m[Q]) ? a.d.m[Q][(size_t)c.src * w + e] : 0.0f;
    if (a.out_v[Q]) a.out_v[Q][o] = (c.kind == 0 && a.d.v[Q]) ? a.d.v[Q][(size_t)c.src * w + e] : 0.0f;
}

struct GatherGrid { uint32_t start[7]; };

__global__ void __launch_bounds__(256) k_densify_gather(RebuildArgs a, const uint32_t* __restrict__ keep_pos,
                                                        GatherGrid gg) {
    const uint32_t blk = blockIdx.x;
    const uint32_t C = a.d.N + a.nc + a.replicas * a.ns;
    int q = 0;
    while (q < 5 && blk >= gg.start[q + 1]) q++;  // block-uniform
    const uint32_t t = (blk - gg.start[q]) * 256u + threadIdx.x;  // C * width < 2^32 (checked on the host)
    switch (q) {
        case 0: gather_group<0>(a, keep_pos, t, C); break;
        case 1: gather_group<1>(a, keep_pos, t, C); break;
        case 2: gather_group<2>(a, keep_pos, t, C); break;
        case 3: gather_group<3>(a, keep_pos, t, C); break;
        case 4: gather_group<4>(a, keep_pos, t, C); break;
        default: gather_group<5>(a, keep_pos, t, C); break;
    }
}

// Parameter activations of GaussianSplatModel (gaussian_splat_model.py get_opacity / get_scaling / get_quaternion:
// sigmoid, exp, F.normalize(eps 1e-12)) and their backward, one thread per Gaussian, one launch each way (torch
// runs ~4 kernels forward and ~8 backward for the three).
__global__ void __launch_bounds__(256) k_activate_fwd(uint32_t N, const float* __restrict__ ro,
                                                      const float* __restrict__ rs, const float* __restrict__ rq,
                                                      float* __restrict__ o, float* __restrict__ sc,
                                                      float* __restrict__ q, uint64_t* __restrict__ zero_stamp,
                                                      uint64_t stamp) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= N) return;
    o[i] = 1.0f / (1.0f + expf(-ro[i]));
    bool zero = false;
    for (int k = 0; k < 3; k++) {
        const float e = expf(rs[3 * (size_t)i + k]);
        sc[3 * (size_t)i + k] = e;
        zero |= e == 0.0f;
    }
    if (zero && zero_stamp) *zero_stamp = stamp;  // same value from every writer
    const float4 x = reinterpret_cast<const float4*>(rq)[i];
    const float d = fmaxf(sqrtf((x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w)), 1e-12f);
    reinterpret_cast<float4*>(q)[i] = make_float4(x.x / d, x.y / d, x.z / d, x.w / d);
}
__global__ void __launch_bounds__(256) k_activate_bwd(uint32_t N, const float* __restrict__ o,
                                                      const float* __restrict__ sc, const float* __restrict__ rq,
                                                      const float* __restrict__ go, const float* __restrict__ gs_,
                                                      const float* __restrict__ gq, float* __restrict__ dro,
                                                      float* __restrict__ drs, float* __restrict__ drq,
                                                      float scale_reg, const uint64_t* __restrict__ zero_stamp,
                                                      uint64_t stamp) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= N) return;
    dro[i] = go ? sigmoid_bwd(go[i], o[i]) : 0.0f;
    const float* sv = sc + 3 * (size_t)i;
    const int zmode = zero_stamp ? (*zero_stamp == stamp ? 1 : 0) : -1;
    for (int k = 0; k < 3; k++)
        drs[3 * (size_t)i + k] = (gs_ || scale_reg != 0.0f) ? exp_bwd(gs_ ? gs_[3 * (size_t)i + k] : 0.0f, sv, k,
                                                                         scale_reg, zmode)
                                                              : 0.0f;
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gq) r = normalize_bwd(reinterpret_cast<const float4*>(rq)[i], reinterpret_cast<const float4*>(gq)[i]);
    reinterpret_cast<float4*>(drq)[i] = r;
}

// The photometric L1 term of a training view (gaussian_trainer.py: image = render(...).clamp(0, 1), l1_loss =
// |image - gt|.mean()): the clamped image and per-block partial sums of |image - gt| in one pass (the caller sums
// the partials, a fixed order); backward d_img = (g_image + g_l1 sgn(image - gt) / n) [0 <= img <= 1] in one pass
// -- torch runs four kernels forward and five backward for it.
constexpr int L1_PER_THREAD = 16;  // 4 float4 per thread, 4096 floats per block
// torch.clamp(x, 0, 1) keeps NaN (fminf/fmaxf alone would turn it into 0 and hide a diverged render from the loss)
__device__ __forceinline__ float clamp01(float x) { return x != x ? x : fminf(fmaxf(x, 0.f), 1.f); }
__global__ void __launch_bounds__(256) k_clamp_l1_fwd(uint32_t n, const float* __restrict__ img,
                                                      const float* __restrict__ gt, float* __restrict__ out,
                                                      float* __restrict__ partial) {
    __shared__ float s_w[4];
    const size_t base = (size_t)blockIdx.x * 256u * L1_PER_THREAD;
    float acc = 0.0f;
#pragma unroll
    for (int r = 0; r < L1_PER_THREAD / 4; r++) {
        const size_t i = base + ((size_t)r * 256u + threadIdx.x) * 4u;
        if (i + 3 < n) {
            const float4 x = *reinterpret_cast<const float4*>(img + i);
            const float4 g = *reinterpret_cast<const float4*>(gt + i);
            const float4 c = make_float4(clamp01(x.x), clamp01(x.y), clamp01(x.z), clamp01(x.w));
            *reinterpret_cast<float4*>(out + i) = c;
            acc += (fabsf(c.x - g.x) + fabsf(c.y - g.y)) + (fabsf(c.z - g.z) + fabsf(c.w - g.w));
        } else {
            for (size_t j = i; j < n && j < i + 4; j++) {
                const float c = clamp01(img[j]);
                out[j] = c;
                acc += fabsf(c - gt[j]);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}
__global__ void __launch_bounds__(256) k_clamp_l1_bwd(uint32_t n, const float* __restrict__ img,
                                                      const float* __restrict__ clamped, const float* __restrict__ gt,
                                                      const float* __restrict__ g_img, const float* __restrict__ g_l1,
                                                      float g_l1_value, float* __restrict__ d_img) {
    const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    // the L1 term's incoming gradient: a device scalar (autograd) or a value (the native step; 0 = no L1 term)
    const float s = (g_l1 ? g_l1[0] : g_l1_value) / (float)n;
    // the clamped value is recomputed from img (clamp01 is exact): one 4-B read per pixel fewer than loading `clamped`
    const float x = img[i], d = clamp01(x) - gt[i];
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    const float g = (g_img ? g_img[i] : 0.f) + s * sg;
    d_img[i] = (x >= 0.f && x <= 1.f) ? g : 0.f;
}

// torch.prod(x, dim=1) of x [N, M], M <= 3 (the scale regulariser's prod of the scaling), and its autograd backward
// (FunctionsManual.cpp prod_backward) without the host read: torch counts the zeros of x, reads the count back and
// picks dprod * (prod / x) when there are none, else for EVERY row the zero-safe dprod * (exclusive left cumprod x
// exclusive right cumprod).  Here the forward writes the call's stamp to *zero_stamp when some element is 0 and the
// backward compares it with the same stamp, on the device.
// Row order: torch's reduction gives a row of M <= 4 elements to 4 lanes (identity 1 past M) and combines them with
// shuffles at offsets 2 then 1, so the product is (x0 x2)(x1 x3): (x0 x2) x1 for M = 3 (tools/prod_order_probe.py
// finds no other order matching on the GPU).  Every cumprod entry of the zero-safe form has at most two factors
// for M <= 3, so its value does not depend on the scan's association.
__global__ void __launch_bounds__(256) k_row_prod_fwd(uint32_t N, uint32_t M, const float* __restrict__ x,
                                                      float* __restrict__ prod, uint32_t* __restrict__ zero_stamp,
                                                      uint32_t stamp) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    bool z = false;
    if (i < N) {
        const float* r = x + (size_t)i * M;
        const float a = r[0], b = M > 1 ? r[1] : 1.0f, c = M > 2 ? r[2] : 1.0f;
        prod[i] = (a * c) * b;
        z = a == 0.0f || b == 0.0f || c == 0.0f;
    }
    // the call's stamp, not a flag: the word needs no zeroing launch before the forward, and a stale value (another
    // call's stamp) reads as "no zero" in the backward, which compares with its own call's stamp
    if (__any(z) && (threadIdx.x & 63) == 0) *zero_stamp = stamp;  // every lane is live here (no early return)
}
__global__ void __launch_bounds__(256) k_row_prod_bwd(uint32_t N, uint32_t M, const float* __restrict__ x,
                                                      const float* __restrict__ prod, const float* __restrict__ dprod,
                                                      const uint32_t* __restrict__ zero_stamp, uint32_t stamp,
                                                      float* __restrict__ dx) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= N) return;
    const float* r = x + (size_t)i * M;
    float* d = dx + (size_t)i * M;
    const float g = dprod[i];
    if (*zero_stamp != stamp) {
        const float p = prod[i];
        for (uint32_t k = 0; k < M; k++) d[k] = g * (p / r[k]);
        return;
    }
    // cat([1, x0 .. x(M-2)]).cumprod() and cat([1, x(M-1) .. x1]).cumprod().flip()
    float left[3], right[3];
    left[0] = 1.0f;
    for (uint32_t k = 1; k < M; k++) left[k] = left[k - 1] * r[k - 1];
    right[M - 1] = 1.0f;
    for (int k = (int)M - 2; k >= 0; k--) right[k] = right[k + 1] * r[k + 1];
    for (uint32_t k = 0; k < M; k++) d[k] = g * (left[k] * right[k]);
}

}  // namespace

void launch_adam_multi(const AdamMultiArgs& a0, hipStream_t s) {
    AdamMultiArgs a = a0;
    // start[] in blocks: each group gets ceil(N*M / 4 / 256) blocks, the statistics ceil(N / 256)
    uint32_t b = 0;
    for (int k = 0; k < a.n; k++) {
        a.start[k] = b;
        const uint64_t items = ((uint64_t)a.N * a.g[k].M + 3) / 4;  // float4 chunks
        b += (uint32_t)((items + 256 * ADAM_CHUNKS - 1) / (256 * ADAM_CHUNKS));
    }
    a.start[a.n] = b;
    if (a.radii || a.status_out) b += (a.N + 255) / 256;
    if (b == 0) return;
    a.nblocks = b;
    k_adam_multi<<<a.grid_cap && a.grid_cap < b ? a.grid_cap : b, 256, 0, s>>>(a);
}

void launch_densify_select(const DensifyArgs& a, hipStream_t s) {
    if (a.N) k_densify_select<<<(a.N + 255) / 256, 256, 0, s>>>(a);
}
void launch_densify_lists(const DensifyArgs& a, const uint32_t* clone_pos, const uint32_t* split_pos,
                          uint32_t* clone_idx, uint32_t* split_idx, hipStream_t s) {
    if (a.N) k_densify_lists<<<(a.N + 255) / 256, 256, 0, s>>>(a, clone_pos, split_pos, clone_idx, split_idx);
}
void launch_densify_keep(const RebuildArgs& a, hipStream_t s) {
    const uint32_t C = a.d.N + a.nc + a.replicas * a.ns;
    if (C) k_densify_keep<<<(C + 255) / 256, 256, 0, s>>>(a);
}
void launch_densify_gather(const RebuildArgs& a, const uint32_t* keep_pos, hipStream_t s) {
    const uint64_t C = (uint64_t)a.d.N + a.nc + (uint64_t)a.replicas * a.ns;
    GatherGrid gg;
    uint32_t b = 0;
    for (int q = 0; q < 6; q++) {
        gg.start[q] = b;
        b += (uint32_t)((C * a.d.width[q] + 255) / 256);
    }
    gg.start[6] = b;
    if (b) k_densify_gather<<<b, 256, 0, s>>>(a, keep_pos, gg);
}

void launch_activate_fwd(uint32_t N, const float* ro, const float* rs, const float* rq, float* o, float* sc, float* q,
                         uint64_t* zero_stamp, uint64_t stamp, hipStream_t s) {
    if (N) k_activate_fwd<<<(N + 255) / 256, 256, 0, s>>>(N, ro, rs, rq, o, sc, q, zero_stamp, stamp);
}
void launch_activate_bwd(uint32_t N, const float* o, const float* sc, const float* rq, const float* go,
                         const float* gsc, const float* gq, float* dro, float* drs, float* drq, hipStream_t s,
                         float scale_reg, const uint64_t* zero_stamp, uint64_t stamp) {
    if (N)
        k_activate_bwd<<<(N + 255) / 256, 256, 0, s>>>(N, o, sc, rq, go, gsc, gq, dro, drs, drq, scale_reg, zero_stamp,
                                                        stamp);
}

void launch_row_prod_fwd(uint32_t N, uint32_t M, const float* x, float* prod, uint32_t* zero_stamp, uint32_t stamp,
                         hipStream_t s) {
    if (N) k_row_prod_fwd<<<(N + 255) / 256, 256, 0, s>>>(N, M, x, prod, zero_stamp, stamp);
}
void launch_row_prod_bwd(uint32_t N, uint32_t M, const float* x, const float* prod, const float* dprod,
                         const uint32_t* zero_stamp, uint32_t stamp, float* dx, hipStream_t s) {
    if (N) k_row_prod_bwd<<<(N + 255) / 256, 256, 0, s>>>(N, M, x, prod, dprod, zero_stamp, stamp, dx);
}

uint32_t clamp_l1_blocks(uint32_t n) { return (n + 256u * L1_PER_THREAD - 1) / (256u * L1_PER_THREAD); }
void launch_clamp_l1_fwd(uint32_t n, const float* img, const float* gt, float* out, float* partial, hipStream_t s) {
    if (n) k_clamp_l1_fwd<<<clamp_l1_blocks(n), 256, 0, s>>>(n, img, gt, out, partial);
}
void launch_clamp_l1_bwd(uint32_t n, const float* img, const float* clamped, const float* gt, const float* g_img,
                         const float* g_l1, float* d_img, hipStream_t s, float g_l1_value) {
    if (n) k_clamp_l1_bwd<<<(n + 255) / 256, 256, 0, s>>>(n, img, clamped, gt, g_img, g_l1, g_l1_value, d_img);
}

// Sum of x[0..n) (mode 0) or of the row products (x[3i] x[3i+2]) x[3i+1] over n rows (mode 1: the scale
// regulariser's prod(scaling, 1)) into one partial per 256-thread block; k_loss_final totals the partials in order.
__global__ void __launch_bounds__(256) k_block_sum(const float* __restrict__ x, uint32_t n, int mode,
                                                   float* __restrict__ partial) {
    __shared__ float s_w[4];
    float acc = 0.0f;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
        acc += mode ? (x[3 * (size_t)i] * x[3 * (size_t)i + 2]) * x[3 * (size_t)i + 1] : x[i];  // torch.prod's order
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}
// loss[0] = L1 (mean |clamped - gt|), loss[1] = SSIM (mean of the map), loss[2] = mean prod(scaling, 1); one
// 1024-thread block, fixed summation order (strided per thread, then the waves, then the 16 wave sums in order)
__global__ void __launch_bounds__(1024) k_loss_final(const float* __restrict__ p_l1, uint32_t n_l1,
                                                     const float* __restrict__ p_ssim, uint32_t n_ssim,
                                                     const float* __restrict__ p_sc, uint32_t n_sc, uint32_t n_img,
                                                     uint32_t P, float* __restrict__ loss) {
    __shared__ float s_w[3][16];
    const float* ps[3] = {p_l1, p_ssim, p_sc};
    const uint32_t ns[3] = {n_l1, n_ssim, n_sc};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float acc = 0.0f;
        for (uint32_t i = threadIdx.x; i < ns[k]; i += 1024) acc += ps[k][i];
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if ((threadIdx.x & 63) == 0) s_w[k][threadIdx.x >> 6] = acc;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int k = threadIdx.x;
        float acc = 0.0f;
        for (int w = 0; w < 16; w++) acc += s_w[k][w];
        loss[k] = acc / (float)(k == 2 ? P : n_img);
    }
}
uint32_t block_sum_blocks(uint32_t n) {
    const uint32_t b = (n + 255) / 256;
    return b < 1024u ? (b ? b : 1u) : 1024u;
}
void launch_block_sum(const float* x, uint32_t n, int mode, float* partial, hipStream_t s) {
    k_block_sum<<<block_sum_blocks(n), 256, 0, s>>>(x, n, mode, partial);
}
void launch_loss_final(const float* p_l1, uint32_t n_l1, const float* p_ssim, uint32_t n_ssim, const float* p_sc,
                       uint32_t n_sc, uint32_t n_img, uint32_t P, float* loss, hipStream_t s) {
    k_loss_final<<<1, 1024, 0, s>>>(p_l1, n_l1, p_ssim, n_ssim, p_sc, n_sc, n_img, P, loss);
}

}  // namespace gs

// raster_bwd.hip -- backward of the tile rasterizer for gfx950.
//
// k_render_bwd   one wave64 per tile, 4 pixels per lane, front-to-back replay from T = 1 up to the tile's
//                max contributor. The reference (backward.cu:455-658) replays 32-splat buckets from
//                ~2 GB of sampled forward state; here the state is recomputed on the fly, which is the
//                same arithmetic (T *= 1 - alpha, ar += w c) without the sampled-state traffic.
//                Per splat, the 10 gradient moments are summed over the wave with a transpose
//                reduce-scatter (13 cross-lane exchanges instead of 60) and stored once as a 48-B record
//                at the instance's emission slot -- no float atomics (the chip-wide atomic rate and the
//                scattered-row penalty make per-instance atomicAdd the wrong tool on MI355X).
// k_gauss_sum    a wave per chunk of instance slots sums the records of the Gaussians beginning there
//                (segmented scan, deterministic order) and lists the contributing ones; extra blocks write the
//                view depth (and zero-fill the gradient outputs when the replay could not);
// k_gauss_live   one thread per contributing Gaussian turns the summed moments into dL/d(mean2D, conic,
//                opacity), then computeCov2DCUDA + preprocessCUDA backward (backward.cu:149-451) fused in one pass.
#include <hip/hip_runtime.h>
#include "gs_common.h"
#include "raster.h"
#include "wave_sort.h"

namespace gs {

#ifdef DG_BWD_STATS  // measurement build only: replay utilisation counters, printed per backward by k_bwd_stats_dump
__device__ unsigned long long g_bs[256 * 4];
#endif

__device__ __forceinline__ float bcastf(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float pl32_sum(float a, float b) {  // lane<32: a[l]+a[l+32]; lane>=32: b[l-32]+b[l]
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pl16_sum(float a, float b) {  // even rows: a[l]+a[l+16]; odd rows: b[l-16]+b[l]
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Sum 10 per-lane values over the wave64 as a reduce-scatter: lane-half swap (v_permlane32_swap),
// row swap (v_permlane16_swap), row_mirror / row_half_mirror / quad_perm DPP adds -- 26 VALU ops, no LDS.
// Returns the total of slot `slot` (valid when slot >= 0; one lane per slot writes).
__device__ __forceinline__ float wave_reduce10(const float (&p)[10], int lane, int& slot) {
    const bool b4 = lane & 16, b3 = lane & 8, b2 = lane & 4;
    float q[5];
#pragma unroll
    for (int i = 0; i < 5; i++) q[i] = pl32_sum(p[i], p[5 + i]);         // slot (b5 ? 5 : 0) + i
    float r[3];
    r[0] = pl16_sum(q[0], q[3]);                                         // q-index (b4 ? 3 : 0) + i
    r[1] = pl16_sum(q[1], q[4]);
    r[2] = pl16_sum(q[2], 0.0f);
    const float x0 = r[0] + dpp<0x140>(r[0]);                            // row_mirror: partner l ^ 15
    const float x1 = r[1] + dpp<0x140>(r[1]);
    const float x2 = r[2] + dpp<0x140>(r[2]);
    const float s0 = b3 ? x2 : x0;                                       // r-index (b3 ? 2 : 0) + i
    const float s1 = b3 ? 0.0f : x1;
    const float y0 = s0 + dpp<0x141>(s0);                                // row_half_mirror: partner l ^ 7
    const float y1 = s1 + dpp<0x141>(s1);
    float u = b2 ? y1 : y0;
    u += dpp<0xB1>(u);                                                   // quad_perm [1,0,3,2]
    u += dpp<0x4E>(u);                                                   // quad_perm [2,3,0,1]
    const int ri = (b3 ? 2 : 0) + (b2 ? 1 : 0);
    const bool valid = (ri <= 2) && (!b4 || ri <= 1) && ((lane & 3) == 0);
    slot = valid ? (((lane & 32) ? 5 : 0) + (b4 ? 3 : 0) + ri) : -1;
    return u;
}

// One splat of the replay for the lane's four pixels: exponent, acceptance, the regrouped dL/dalpha terms, the 10
// moments and their wave reduction into the instance's record.  PER_SPLAT_LAST: test "splat index < last contributor"
// per pixel; otherwise athr already holds it (1/255 alive, 2 dead).
template <bool HAS_INVD, bool HAS_BG, bool PER_SPLAT_LAST>
__device__ __forceinline__ void replay_splat(const RenderBwdArgs& a, const float4* sb, int jj, int sidx, const v4f pxv,
                                             const v2f pyv, const int (&last)[4], const v4f athr, const v4f g0,
                                             const v4f g1, const v4f g2, const v4f gd, const v4f ntb, v4f& T, v4f& S,
                                             int lane, uint32_t E1, uint8_t* flag2m) {
    const float4 Sa = sb[jj * 3 + 0], Sb = sb[jj * 3 + 1], Sc = sb[jj * 3 + 2];
    const float sx = Sa.x, sy = Sa.y, so = Sb.y, sr = Sb.z, sg = Sb.w, sbl = Sc.x, si = Sc.y;
    // exponent, identical to the forward's splat_power4
    const v2f dy = bc2(sy) - pyv;
    const v4f dx = bc4(sx) - pxv;
    const v2f bdy = bc2(Sa.w) * dy, cdy2 = (bc2(Sb.x) * dy) * dy;
    const v4f p2 = fma4(dx, fma4(bc4(Sa.z), dx, cat4(bdy, bdy)), cat4(cdy2, cdy2));
    const v4f G = {__builtin_amdgcn_exp2f(p2.x), __builtin_amdgcn_exp2f(p2.y), __builtin_amdgcn_exp2f(p2.z),
                   __builtin_amdgcn_exp2f(p2.w)};
    v4f al = bc4(so) * G;
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float ak = fminf(0.99f, al[k]);
        ok[k] = PER_SPLAT_LAST ? (sidx < last[k]) && !(p2[k] > 0.0f) && !(ak < athr[k])
                               : !(p2[k] > 0.0f) && !(ak < athr[k]);
        al[k] = ok[k] ? ak : 0.0f;
    }
    const v4f wgt = al * T;
    const v4f oma = bc4(1.0f) - al;
    const v4f inv = {__builtin_amdgcn_rcpf(oma.x), __builtin_amdgcn_rcpf(oma.y), __builtin_amdgcn_rcpf(oma.z),
                     __builtin_amdgcn_rcpf(oma.w)};
    v4f cg = fma4(bc4(sbl), g2, fma4(bc4(sg), g1, bc4(sr) * g0));
    if (HAS_INVD) cg = fma4(bc4(si), gd, cg);
    S = fma4(wgt, cg, S);
    v4f dLda = fma4(cg, T, inv * S);
    if (HAS_BG) dLda = fma4(ntb, inv, dLda);
#pragma unroll
    for (int k = 0; k < 4; k++) dLda[k] = ok[k] ? dLda[k] : 0.0f;
    T = T * oma;
    // per-splat moments over the lane's 4 pixels; lo + hi of a v4 = the two row sums {row A, row B}.  A sum of
    // products folds its hi half in with an fma (one packed op fewer per moment than product, product, add).
    const v4f t4 = G * dLda;
    const v4f tdx = t4 * dx;
    const v2f rt = lo2(t4) + hi2(t4);
    const v2f rtx = lo2(tdx) + hi2(tdx);
    const v2f rtxx = fma2(hi2(tdx), hi2(dx), lo2(tdx) * lo2(dx));
    const v2f rc0 = fma2(hi2(wgt), hi2(g0), lo2(wgt) * lo2(g0));
    const v2f rc1 = fma2(hi2(wgt), hi2(g1), lo2(wgt) * lo2(g1));
    const v2f rc2 = fma2(hi2(wgt), hi2(g2), lo2(wgt) * lo2(g2));
    const v2f u = rt * dy;  // {tA dyA, tB dyB}
    float p[10];
    p[0] = rtx.x + rtx.y;                            // SGx
    p[1] = u.x + u.y;                                // SGy
    p[2] = rtxx.x + rtxx.y;                          // SGxx
    p[3] = fmaf(rtx.x, dy.x, rtx.y * dy.y);          // SGxy
    p[4] = fmaf(u.x, dy.x, u.y * dy.y);              // SGyy
    p[5] = rt.x + rt.y;                              // SG
    p[6] = rc0.x + rc0.y;
    p[7] = rc1.x + rc1.y;
    p[8] = rc2.x + rc2.y;
    if (HAS_INVD) {
        const v2f rcd = fma2(hi2(wgt), hi2(gd), lo2(wgt) * lo2(gd));
        p[9] = rcd.x + rcd.y;
    } else {
        p[9] = 0.0f;
    }
#ifdef DG_BWD_STATS
    {
        const uint32_t nok = (uint32_t)__popcll(__ballot(ok[0])) + (uint32_t)__popcll(__ballot(ok[1])) +
                             (uint32_t)__popcll(__ballot(ok[2])) + (uint32_t)__popcll(__ballot(ok[3]));
        if (lane == 0) {
            const uint32_t b = (uint32_t)(blockIdx.x & 255u) * 4u;
            atomicAdd(&g_bs[b + 0], 1ull);
            atomicAdd(&g_bs[b + 1], nok ? 1ull : 0ull);
            atomicAdd(&g_bs[b + 2], (unsigned long long)nok);
        }
    }
#endif
    if (__any(ok[0] || ok[1] || ok[2] || ok[3])) {
        int slot;
        const float tot = wave_reduce10(p, lane, slot);
        const uint32_t e = __builtin_amdgcn_readfirstlane(__float_as_uint(Sc.z));
        if (slot >= 0) a.rec[(size_t)e * REC_STRIDE + slot] = tot;
        if (lane == 0) (e < E1 ? a.flag : flag2m)[e] = 1;  // phase-2 flags: flag2[e - E1]
    }
}

// Front-to-back replay.  Lane l owns pixels (l&7, l>>3) and (l&7 + 8, l>>3) of the tile's top half
// (pair A = quadrants 0,1) and the same two of the bottom half (pair B = quadrants 2,3); each pair is
// one row, evaluated with packed fp32.  Per 64-splat batch each lane stages its splat in wave-private
// LDS with a 4-bit mask of the quadrants it can touch (quad_mask) that still have pixels before their
// last contributor; the wave walks only splats with a non-empty mask and skips a pair whose two mask
// bits are clear (wave-uniform branch).  Inactive (pixel, splat) pairs get alpha = 0, dL/dalpha = 0.
//
// The per-pixel gradient terms of backward.cu:600-650 are regrouped so that everything constant per
// splat leaves the pixel loop (exact algebra, fp32 rounding differs from the per-term sums):
//   dL/dalpha = T (c.g) + (ar.g)/(1 - alpha) [- T_final (bg.g)/(1 - alpha)]   g = dL/dpixel (+ invdepth)
//   with S = ar.g carried as ONE scalar per pixel (S += w (c.g)) instead of 3-4 channel accumulators,
// and with t = G dL/dalpha the splat's sums reduce to the moments
//   SG = sum t, SGx = sum t dx, SGy = sum t dy, SGxx = sum t dx^2, SGxy = sum t dx dy, SGyy = sum t dy^2
// from which k_gauss_bwd forms dL/dmean2D = -(W/2, H/2) o (a SGx + b SGy, c SGy + b SGx),
// dL/dconic = -o/2 (SGxx, SGxy, SGyy) and dL/dopacity = SG once per Gaussian (the map is linear, so
// summing the moments over instances first is exact).
// Record slots: 0 SGx, 1 SGy, 2 SGxx, 3 SGxy, 4 SGyy, 5 SG, 6-8 sum w g_rgb, 9 sum w g_invdepth.
template <bool HAS_INVD, bool HAS_BG>
__device__ __forceinline__ void render_bwd_tile(const RenderBwdArgs& a, int tile, int lane, float4* sb) {
    // the tile's list = its phase-1 prefix followed by its phase-2 remainder (depth-prefix binning)
    const uint2 rg = a.ranges[tile];
    const int n1 = (int)(rg.y - rg.x);
    uint2 rg2 = make_uint2(0u, 0u);
    if (a.ranges2 && a.unfinished[tile]) rg2 = a.ranges2[tile];
    const int nall = n1 + (int)(rg2.y - rg2.x);
    const uint32_t E1 = a.counters[CNT_E1];
    uint8_t* const flag2m = a.flag2 ? a.flag2 - E1 : a.flag;
    const int mc = (int)a.max_contrib[tile];
    const int n = nall < mc ? nall : mc;
    if (n <= 0) return;
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int tx0 = tx * GS_TILE_X, ty0 = ty * GS_TILE_Y;
    const size_t HW = (size_t)a.W * a.H;
    const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
    // pixel k of the lane: column c0 + 8 (k >> 1), row rA + 8 (k & 1) -- the forward's layout
    const int c0 = tx0 + (lane & 7), rA = ty0 + (lane >> 3);
    const v4f pxv = {(float)c0, (float)c0, (float)(c0 + 8), (float)(c0 + 8)};
    const v2f pyv = {(float)rA, (float)(rA + 8)};
    v4f T = bc4(1.0f), S, g0, g1, g2, gd, ntb;
    int last[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int px = c0 + (k >> 1) * 8, py = rA + (k & 1) * 8;
        if (px < a.W && py < a.H) {
            const size_t pid = (size_t)py * a.W + px;
            last[k] = (int)a.n_contrib[pid];
            g0[k] = a.dL_dpix[pid]; g1[k] = a.dL_dpix[HW + pid]; g2[k] = a.dL_dpix[2 * HW + pid];
            gd[k] = HAS_INVD ? a.dL_dinvd[pid] : 0.0f;
            // ar starts at -(final pixel colour) (backward.cu:538-546); S = ar . g
            float s0 = -(fmaf(a.img_color[2 * HW + pid], g2[k], fmaf(a.img_color[HW + pid], g1[k], a.img_color[pid] * g0[k])));
            if (HAS_INVD) s0 = fmaf(-a.img_invd[pid], gd[k], s0);
            S[k] = s0;
            ntb[k] = HAS_BG ? -a.final_T[pid] * fmaf(bg2, g2[k], fmaf(bg1, g1[k], bg0 * g0[k])) : 0.0f;
        } else {
            last[k] = 0;
            S[k] = g0[k] = g1[k] = g2[k] = gd[k] = ntb[k] = 0.0f;
        }
    }
    // per quadrant (qx = k >> 1, qy = k & 1 -> quadrant 2 qy + qx): max last contributor over the wave
    int qlast[4];
#pragma unroll
    for (int k = 0; k < 4; k++) qlast[2 * (k & 1) + (k >> 1)] = (int)wave_max_u32((uint32_t)last[k]);
#ifndef DG_BWD_NO_PREFETCH
    // The batch gather is a dependent chain (list slot -> emission index -> Gaussian -> splat record).  The first two
    // links of batch b + 1 (and the first of b + 2) are loaded while batch b replays, so a batch start waits on one
    // HBM round trip instead of three.
    auto slot_of = [&](int j) -> uint32_t {  // emission index of list position j (phase-2 entries: local index)
        if (j >= n) return 0u;
        return j < n1 ? min(a.s_e[rg.x + j], a.K1 - 1) : min(a.s_e2[rg2.x + (uint32_t)(j - n1)], a.K - 1 - E1);
    };
    auto gauss_of = [&](int j, uint32_t e) -> uint32_t {
        if (j >= n) return 0u;
        return j < n1 ? min(a.eg[e], a.P - 1) : min(a.eg2[e], a.P - 1);
    };
    uint32_t e_cur = slot_of(lane), e_nxt = slot_of(64 + lane);
    uint32_t g_cur = gauss_of(lane, e_cur);
#endif
    for (int base = 0; base < n; base += 64) {
        const int j = base + lane;
        uint32_t qm = 0;
#ifndef DG_BWD_NO_PREFETCH
        const uint32_t ee_b = j < n1 ? e_cur : E1 + e_cur, g_b = g_cur;
        if (base + 64 < n) {
            g_cur = gauss_of(j + 64, e_nxt);
            e_cur = e_nxt;
            e_nxt = slot_of(j + 128);
        }
#endif
        if (j < n) {
#ifndef DG_BWD_NO_PREFETCH
            const uint32_t ee = ee_b, g = g_b;
#else
            uint32_t ee, g;
            if (j < n1) {
                ee = min(a.s_e[rg.x + j], a.K1 - 1);
                g = min(a.eg[ee], a.P - 1);
            } else {
                const uint32_t el = min(a.s_e2[rg2.x + (uint32_t)(j - n1)], a.K - 1 - E1);
                ee = E1 + el;
                g = min(a.eg2[el], a.P - 1);
            }
#endif
            const float4 s0 = a.sp[2 * g], s1 = a.sp[2 * g + 1];
            const float2 m = make_float2(s0.x, s0.y);
            const float4 c4 = make_float4(s0.z, s0.w, s1.x, s1.y);
            const float4 q = a.rgbi[g];
            const float thr = quad_log_thr(c4.w);
            qm = quad_mask({c4.x, c4.y, c4.z, c4.w}, m.x, m.y, thr, tx0, ty0);
#pragma unroll
            for (int k = 0; k < 4; k++) qm &= (j < qlast[k]) ? 0xfu : ~(1u << k);
            const SplatExp kq = splat_exp_coeffs(c4.x, c4.y, c4.z);
            sb[lane * 3 + 0] = make_float4(m.x, m.y, kq.A, kq.B);
            sb[lane * 3 + 1] = make_float4(kq.C, c4.w, q.x, q.y);
            sb[lane * 3 + 2] = make_float4(q.z, q.w, __uint_as_float(ee), 0.0f);
        }
        __builtin_amdgcn_wave_barrier();
        uint64_t smask = __ballot(qm != 0u);
#ifndef DG_BWD_NO_BATCH_ALIVE
        // A pixel's last contributor lies inside this batch for few pixels: when it lies outside for every pixel of
        // the wave, "splat index < last" is constant over the batch and folds into the acceptance threshold (2 > any
        // alpha: dead), as the forward's; otherwise the per-splat test.
        bool straddle = false;
#pragma unroll
        for (int k = 0; k < 4; k++) straddle |= last[k] > base && last[k] < base + 64;
        if (!__any(straddle)) {
            v4f athr;
#pragma unroll
            for (int k = 0; k < 4; k++) athr[k] = last[k] > base ? (1.0f / 255.0f) : 2.0f;
            while (smask) {
                const int jj = (int)__builtin_ctzll(smask);
                smask &= smask - 1;
                replay_splat<HAS_INVD, HAS_BG, false>(a, sb, jj, base + jj, pxv, pyv, last, athr, g0, g1, g2, gd, ntb, T, S,
                                                       lane, E1, flag2m);
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
#endif
        while (smask) {
            const int jj = (int)__builtin_ctzll(smask);
            smask &= smask - 1;
            replay_splat<HAS_INVD, HAS_BG, true>(a, sb, jj, base + jj, pxv, pyv, last, bc4(1.0f / 255.0f), g0, g1, g2, gd,
                                                 ntb, T, S, lane, E1, flag2m);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Replay length of a tile: its list (phase 1 + phase 2) cut at the last contributor, as render_bwd_tile.
// Replay length of a tile for the launch order: its max contributor (the replay runs to it; the list is never
// shorter), one load per tile.
__device__ __forceinline__ uint32_t replay_len(const RenderBwdArgs& a, int tile) { return a.max_contrib[tile]; }

// Longest-first launch order for the replay (tile_order_sort: the phase-2 emission's extra block, else k_bwd_order).  Per tile, not per 4-tile block:
// ordering whole blocks by their longest tile measured 6% slower.

#ifdef DG_BWD_WPE  // occupancy experiment: cap VGPRs so that DG_BWD_WPE waves fit per SIMD
#define BWD_WPE_ATTR __attribute__((amdgpu_waves_per_eu(DG_BWD_WPE)))
#else
#define BWD_WPE_ATTR
#endif
__global__ void __launch_bounds__(256) BWD_WPE_ATTR k_render_bwd(RenderBwdArgs a) {
    __shared__ float4 s_b[4][64][3];
    const int lane = threadIdx.x & 63;
    // The replay is VALU-bound and leaves HBM mostly idle: each wave zero-fills its share of the gradient outputs
    // (fire-and-forget 16-B stores) for the per-Gaussian pass, which then writes only the contributing Gaussians.
    // Shares are whole 1-KiB chunks, so every store is aligned.
    auto zero_share = [&]() {
        if (!a.zero_base) return;
        // only the first 3/4 of the launch order (the longer replays, longest first) fill, so the kernel's tail has no
        // store drain (render_bwd 257-260 -> 255-258 us, profiles/r03al_bwd_fill_front_ab.txt)
        const size_t nw_all = (size_t)gridDim.x * 4, gw = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
#ifndef DG_BWD_FILL_FRAC4
#define DG_BWD_FILL_FRAC4 3
#endif
        const size_t nw = nw_all * DG_BWD_FILL_FRAC4 / 4 > 0 ? nw_all * DG_BWD_FILL_FRAC4 / 4 : 1;
        if (gw >= nw) return;
        const size_t n4 = a.zero_count / 4;
        const size_t per = ((n4 + nw - 1) / nw + 63) & ~(size_t)63;
        // non-temporal (streaming) stores: ~284 MB of zeros per 1e6-Gaussian view that nothing reads back soon
        v4f* z4 = reinterpret_cast<v4f*>(a.zero_base);
        const size_t e4 = (gw + 1) * per < n4 ? (gw + 1) * per : n4;
        for (size_t i = gw * per + lane; i < e4; i += 64) __builtin_nontemporal_store(bc4(0.0f), &z4[i]);
        if (gw == 0)
            for (size_t i = (n4 << 2) + lane; i < a.zero_count; i += 64) a.zero_base[i] = 0.f;
    };
    const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
    // The share goes out after the wave's replay: issued at the start, the first round of waves put ~140 MB of stores
    // in front of their own gathers (render_bwd 275-277 -> 266-267 us per view with the stores at the end,
    // profiles/r03af_bwd_fill_late_ab.txt; DG_BWD_FILL_EARLY restores the start).
#ifdef DG_BWD_FILL_EARLY
    zero_share();
    if (slot >= a.num_tiles) return;
#else
    if (slot >= a.num_tiles) { zero_share(); return; }
#endif
    const int tile = a.order ? (int)a.order[slot] : slot;
    float4* sb = &s_b[threadIdx.x >> 6][0][0];
    const bool has_bg = a.bg[0] != 0.0f || a.bg[1] != 0.0f || a.bg[2] != 0.0f;
    // the inverse-depth terms only where this tile has a nonzero dL/dinvdepth: elsewhere they add exact zeros
    bool invd_nz = false;
    if (a.dL_dinvd) {
        const int tx0 = (tile % a.tiles_x) * GS_TILE_X, ty0 = (tile / a.tiles_x) * GS_TILE_Y;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int px = tx0 + (lane & 7) + (k >> 1) * 8, py = ty0 + (lane >> 3) + (k & 1) * 8;
            if (px < a.W && py < a.H) invd_nz |= a.dL_dinvd[(size_t)py * a.W + px] != 0.0f;
        }
    }
    const bool has_invd = __any(invd_nz);
    if (has_invd) {
        if (has_bg) render_bwd_tile<true, true>(a, tile, lane, sb);
        else render_bwd_tile<true, false>(a, tile, lane, sb);
    } else {
        if (has_bg) render_bwd_tile<false, true>(a, tile, lane, sb);
        else render_bwd_tile<false, false>(a, tile, lane, sb);
    }
#ifndef DG_BWD_FILL_EARLY
    zero_share();
#endif
}

// The replay order when the forward did not compute it (no phase 2: its emission launch carries the order block):
// one 1024-thread block, longest first.  The record flags are zeroed by the forward's emission, and the inverse-depth
// terms are decided per tile by the replay, so nothing else precedes the replay.
__global__ void __launch_bounds__(1024) k_bwd_order(RenderBwdArgs a) {
    tile_order_sort(a.num_tiles, a.order, [&](int tile) { return replay_len(a, tile); });
}

// ---------------------------------------------------------------------------------------------------
// per-Gaussian backward: record sum + computeCov2DCUDA + preprocessCUDA (backward.cu:23-451)
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ float sq(float x) { return x * x; }

__device__ __forceinline__ void gauss_bwd_one(const GaussBwdArgs& a, int idx, const float (&acc)[10]);

// ---- record sum: instance-parallel segmented reduction over the record slots
// The instances of a Gaussian are contiguous slots in Gaussian order (phase 1 in [0, E1), phase 2 after it), and only
// ~5% of the Gaussians have any, so the sum walks the slots, not the Gaussians: a wave per chunk of SUM_CHUNK slots,
// 64 per step (owner, flag and record loads coalesced).  A Gaussian belongs to the chunk holding its first slot; the
// wave skips the slots of a Gaussian begun in the chunk before and follows its last one past the chunk end.  Sums:
// a segmented scan over the lanes (segments = owners) per step, plus the open segment carried from the previous step
// -- a fixed order, deterministic.  The segment's last lane writes the Gaussian's 10 sums and its index over its own
// record (read by now, by this wave only) and appends the slot to the chunk's list if any sum is nonzero.
__device__ __forceinline__ uint32_t inst_owner(const GaussBwdArgs& a, uint32_t e, uint32_t E1) {
    return e < E1 ? a.eg[e] : a.eg2[e - E1];
}
struct SumRange { uint32_t E1, NR; };
__device__ __forceinline__ SumRange sum_range(const GaussBwdArgs& a) {
    SumRange r;
    r.E1 = min(a.counters[CNT_E1], min(a.K1, a.K));
    r.NR = a.eg2 ? min(r.E1 + a.counters[CNT_K2], a.K) : r.E1;
    return r;
}

// A record's 10 floats (REC_STRIDE floats apart: 8-B aligned at 40 B, 16-B aligned at 48 B).
struct Rec10 { float v[10]; };
__device__ __forceinline__ Rec10 load_rec(const float* rec, uint32_t e) {
    Rec10 r;
    const float* p = rec + (size_t)e * REC_STRIDE;
    if (REC_STRIDE == 12) {
        const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
        const float2 c = reinterpret_cast<const float2*>(p)[4];
        r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w; r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
        r.v[8] = c.x; r.v[9] = c.y;
    } else {
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const float2 q = reinterpret_cast<const float2*>(p)[k];
            r.v[2 * k] = q.x; r.v[2 * k + 1] = q.y;
        }
    }
    return r;
}
__device__ __forceinline__ void store_rec(float* rec, uint32_t e, const float (&v)[10]) {
    float* p = rec + (size_t)e * REC_STRIDE;
#pragma unroll
    for (int k = 0; k < 5; k++) reinterpret_cast<float2*>(p)[k] = make_float2(v[2 * k], v[2 * k + 1]);
}

// One 64-slot step: o/f/r are this lane's slot (owner, flag, record; loaded by the caller, unconditionally, so that
// the loads of every step are in flight together), nxt63 the owner of the slot after lane 63's.
struct SumStep {
    float carry[10];
    uint32_t carry_owner, nlive;
};
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void seg_level(uint32_t own, float (&v)[10]) {
    // rows the DPP does not write, and lanes without a source, keep `old`: owner ~0 (never a lane's owner), value 0
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)own, CTRL, ROW_MASK, 0xf, false);
    const bool same = up == own;
    // sum, then select: the DPP move folds into the add (v_add_f32_dpp), two VALU per value instead of three
#pragma unroll
    for (int k = 0; k < 10; k++) {
        const float t = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[k]), CTRL, ROW_MASK, 0xf, false));
        const float s = v[k] + t;
        v[k] = same ? s : v[k];
    }
}
__device__ __forceinline__ bool sum_step(const GaussBwdArgs& a, uint32_t i0, uint32_t lo, uint32_t hi, uint32_t skip,
                                         uint32_t tail, const SumRange R, int lane, uint32_t o, bool f, const Rec10& r,
                                         uint32_t nxt63, SumStep& st) {
    const uint32_t e = i0 + (uint32_t)lane;
    const bool valid = e < R.NR && o != skip && (e < hi || o == tail) && o < (uint32_t)a.P;
    // invalid lanes: a segment of their own (Gaussian ids < 2^31; never equal to carry_owner's ~0)
    const uint32_t own = valid ? o : (0x80000000u | (uint32_t)lane);
    float v[10];
    const bool use = valid && f;
#pragma unroll
    for (int k = 0; k < 10; k++) v[k] = use ? r.v[k] : 0.f;
    // segmented inclusive scan with DPP (no LDS): row_shr 1, 2, 4, 8 within each 16-lane row, then row_bcast:15
    // and row_bcast:31 across rows; a lane adds its partner's partial only when both have the same owner (segments
    // are contiguous, so everything between them does too)
    // a step with no flagged record (more than half the binned Gaussians have no accepted pixel: their instances lie
    // past their tiles' last contributors) scans zeros: +0 everywhere, so the scan is skipped with the same bits
    if (__any(use)) {
        seg_level<0x111, 0xf>(own, v);
        seg_level<0x112, 0xf>(own, v);
        seg_level<0x114, 0xf>(own, v);
        seg_level<0x118, 0xf>(own, v);
        seg_level<0x142, 0xa>(own, v);
        seg_level<0x143, 0xc>(own, v);
    }
    if (own == st.carry_owner) {  // the step's first segment continues the open one
#pragma unroll
        for (int k = 0; k < 10; k++) v[k] += st.carry[k];
    }
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)own, 0x130, 0xf, 0xf, false);  // wave_shl:1
    const bool last = valid && (lane == 63 ? nxt63 != own : dn != own);
    bool live = false;
#pragma unroll
    for (int k = 0; k < 10; k++) live |= v[k] != 0.0f;
    live = live && last;
    const uint64_t lm = __ballot(live);
    if (live) {
        store_rec(a.rec, e, v);
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        a.live_list[(size_t)lo + st.nlive + (uint32_t)__popcll(lm & lt)] = make_uint2(e, own);
    }
    st.nlive += (uint32_t)__popcll(lm);
    // lane 63's segment stays open when it continues into the next step
    const bool open = __builtin_amdgcn_readlane((int)(valid && !last), 63) != 0;
    st.carry_owner = open ? (uint32_t)__builtin_amdgcn_readlane((int)own, 63) : 0xffffffffu;
#pragma unroll
    for (int k = 0; k < 10; k++) st.carry[k] = bcastf(v[k], 63);
    return open;
}

__device__ __forceinline__ void sum_chunk(const GaussBwdArgs& a, uint32_t ch, const SumRange R, int lane) {
    const uint32_t lo = ch * SUM_CHUNK, hi = min(lo + SUM_CHUNK, R.NR);
    // every load of the chunk's SUM_STEPS + 1 steps (the last one for the tail Gaussian running past hi) is issued
    // before any is used: one HBM round trip per chunk instead of two per step
    constexpr int PF = SUM_STEPS + 1;
    const uint32_t skip = lo ? inst_owner(a, lo - 1, R.E1) : 0xffffffffu;  // begun in the chunk before
    const uint32_t tail = inst_owner(a, hi - 1, R.E1);                      // may run past hi
    uint32_t o[PF];
    bool f[PF];
    Rec10 rr[PF];
#pragma unroll
    for (int q = 0; q < PF; q++) {
        const uint32_t e = lo + 64u * q + (uint32_t)lane;
        o[q] = 0xffffffffu; f[q] = false;
#pragma unroll
        for (int k = 0; k < 10; k++) rr[q].v[k] = 0.f;
        if (e < R.NR) {
            o[q] = inst_owner(a, e, R.E1);
            f[q] = (e < R.E1 ? a.flag[e] : a.flag2[e - R.E1]) != 0;
            rr[q] = load_rec(a.rec, e);
        }
    }
    const uint32_t after = lo + 64u * PF;
    const uint32_t nxt_pf = (lane == 63 && after < R.NR) ? inst_owner(a, after, R.E1) : 0xffffffffu;
    SumStep st;
#pragma unroll
    for (int k = 0; k < 10; k++) st.carry[k] = 0.f;
    st.carry_owner = 0xffffffffu;
    st.nlive = 0;
    bool open = false;
    if (skip != tail) {  // else one Gaussian covers the whole chunk and belongs to an earlier one
        bool done = false;
#pragma unroll
        for (int q = 0; q < PF; q++) {
            if (!done) {
                const uint32_t i0 = lo + 64u * q;
                const uint32_t n63 = q + 1 < PF ? (uint32_t)__builtin_amdgcn_readlane((int)o[q + 1 < PF ? q + 1 : q], 0)
                                                : nxt_pf;
                const uint32_t nx = i0 + 64u < R.NR ? n63 : 0xffffffffu;
                open = sum_step(a, i0, lo, hi, skip, tail, R, lane, o[q], f[q], rr[q], nx, st);
                done = i0 >= R.NR || (i0 + 64u >= hi && !open);
            }
        }
        // a tail Gaussian still open after the prefetched steps: one step at a time
        for (uint32_t i0 = after; open && i0 < R.NR; i0 += 64u) {
            const uint32_t e = i0 + (uint32_t)lane;
            uint32_t oo = 0xffffffffu, n63 = 0xffffffffu;
            bool ff = false;
            Rec10 q;
#pragma unroll
            for (int k = 0; k < 10; k++) q.v[k] = 0.f;
            if (e < R.NR) {
                oo = inst_owner(a, e, R.E1);
                ff = (e < R.E1 ? a.flag[e] : a.flag2[e - R.E1]) != 0;
                q = load_rec(a.rec, e);
                if (lane == 63 && e + 1 < R.NR) n63 = inst_owner(a, e + 1, R.E1);
            }
            open = sum_step(a, i0, lo, hi, skip, tail, R, lane, oo, ff, q, n63, st);
        }
    }
    if (lane == 0) a.live_cnt[ch] = st.nlive;
}

// Gaussians' view depth (the forward's depth key for rendered ones, 0 otherwise) and, when k_render_bwd did not
// zero-fill the nine gradient outputs (not contiguous), their zero fill: one block per AUX_SPAN Gaussians.
constexpr int AUX_SPAN = 1024;
__device__ __forceinline__ void zero_slice(float* out, size_t first, size_t count) {
    float* p = out + first;
    size_t i = threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0u) {
        float4* p4 = reinterpret_cast<float4*>(p);
        for (; i < count / 4; i += 256) p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        i = (count & ~(size_t)3) + threadIdx.x;
    }
    for (; i < count; i += 256) p[i] = 0.f;
}
__device__ __forceinline__ void gauss_aux(const GaussBwdArgs& a, uint32_t blk) {
    const size_t b0 = (size_t)blk * AUX_SPAN;
    const size_t nloc = (size_t)a.P - b0 < (size_t)AUX_SPAN ? (size_t)a.P - b0 : (size_t)AUX_SPAN;
    const size_t M = (size_t)a.M;
    if (!a.outputs_zeroed) {
        zero_slice(a.dmeans2D, 3 * b0, 3 * nloc);
        zero_slice(a.dcolors, 3 * b0, 3 * nloc);
        zero_slice(a.dopacity, b0, nloc);
        zero_slice(a.dmeans3D, 3 * b0, 3 * nloc);
        zero_slice(a.dcov3D, 6 * b0, 6 * nloc);
        zero_slice(a.ddc, 3 * b0, 3 * nloc);
        if (a.dsh && M) zero_slice(a.dsh, 3 * M * b0, 3 * M * nloc);
        zero_slice(a.dscales, 3 * b0, 3 * nloc);
        zero_slice(a.drot, 4 * b0, 4 * nloc);
    }
    for (size_t i = threadIdx.x; i < nloc; i += 256) {
        const size_t idx = b0 + i;
        const uint32_t key = a.dkey[idx];
        a.depth[idx] = (a.radii[idx] > 0 && key != 0xffffffffu) ? __uint_as_float(key) : 0.f;
    }
}

// blocks [0, sum_blocks): record-sum waves (grid-stride over the chunks: phase 2 may add chunks past the phase-1
// capacity the grid is sized for); the rest: gauss_aux.  The zero fill must precede k_gauss_live (next launch).
__global__ void __launch_bounds__(256) k_gauss_sum(GaussBwdArgs a, uint32_t sum_blocks) {
#ifdef DG_SUM_NOAUX  // timing experiment only
    if (blockIdx.x >= sum_blocks) return;
#endif
    if (blockIdx.x >= sum_blocks) {
        gauss_aux(a, blockIdx.x - sum_blocks);
        return;
    }
    const int lane = threadIdx.x & 63;
    const SumRange R = sum_range(a);
    const uint32_t nchunks = (R.NR + SUM_CHUNK - 1) / SUM_CHUNK;
    for (uint32_t ch = blockIdx.x * 4 + (threadIdx.x >> 6); ch < nchunks; ch += sum_blocks * 4)
        sum_chunk(a, ch, R, lane);
}

// LIVE_CHUNKS chunk lists per block (grid-stride), one lane per listed Gaussian (~7 per chunk on the bench scene).
#ifndef DG_LIVE_CHUNKS
#define DG_LIVE_CHUNKS 16
#endif
constexpr int LIVE_CHUNKS = DG_LIVE_CHUNKS;
// the chunk-count prefix below is one wave's scan (64 lanes) and the lookup a binary search over it
static_assert(LIVE_CHUNKS >= 1 && LIVE_CHUNKS <= 64 && (LIVE_CHUNKS & (LIVE_CHUNKS - 1)) == 0,
              "DG_LIVE_CHUNKS: a power of two up to 64");
// threads per block: the listed Gaussians of a block (~2 per chunk) fill about one wave, and the per-Gaussian pass
// needs ~220 VGPRs (2 waves per SIMD), so 256-thread blocks left idle waves holding residency slots.  gauss_bwd per
// view (3 interleaved bench runs each, profiles/r03aa_live_threads_ab.txt): 256 threads 62-63 us, 128: 59, 64: 63-64
#ifndef DG_LIVE_THREADS
#define DG_LIVE_THREADS 128
#endif
constexpr int LIVE_THREADS = DG_LIVE_THREADS;
__global__ void __launch_bounds__(LIVE_THREADS) k_gauss_live(GaussBwdArgs a) {
    __shared__ uint32_t s_pre[LIVE_CHUNKS + 1];
    const SumRange R = sum_range(a);
    const uint32_t nchunks = (R.NR + SUM_CHUNK - 1) / SUM_CHUNK;
    for (uint32_t c0 = blockIdx.x * LIVE_CHUNKS; c0 < nchunks; c0 += gridDim.x * LIVE_CHUNKS) {
        if (threadIdx.x < 64) {
            const uint32_t t = threadIdx.x;
            const uint32_t incl =
                wave_incl_scan((t < (uint32_t)LIVE_CHUNKS && c0 + t < nchunks) ? a.live_cnt[c0 + t] : 0u);
            if (t < (uint32_t)LIVE_CHUNKS) s_pre[t + 1] = incl;
            if (t == 0) s_pre[0] = 0u;
        }
        __syncthreads();
        const uint32_t tot = s_pre[LIVE_CHUNKS];
        for (uint32_t j = threadIdx.x; j < tot; j += LIVE_THREADS) {
            int k = 0;
#pragma unroll
            for (int st = LIVE_CHUNKS / 2; st > 0; st >>= 1)
                if (s_pre[k + st] <= j) k += st;
            const uint2 le = a.live_list[(size_t)(c0 + k) * SUM_CHUNK + (j - s_pre[k])];
            const Rec10 r = load_rec(a.rec, le.x);    // the Gaussian's 10 sums (k_gauss_sum wrote them here)
            gauss_bwd_one(a, (int)min(le.y, (uint32_t)a.P - 1u), r.v);
        }
        __syncthreads();
    }
}

// computeColorFromSH backward (backward.cu:23-144) of one Gaussian; clamped flags recomputed from the forward rgb.
// VEC: degree 3 with 15 rest rows (the bench / training layout), the row read and dL/dsh written with dword-aligned
// dwordx4 accesses (45 dword accesses per lane, each touching its own cache line, made the per-Gaussian pass bound by
// the address units); SHV(k, ch) reads coefficient (k, ch) from registers (VEC) or memory.
template <bool VEC, typename Get>
__device__ __forceinline__ void sh_bwd(const GaussBwdArgs& a, int idx, f3 mean, f3 dcv, const float (&acc)[10],
                                       Get&& SHV, float* dsh_row, f3& dmean) {
    {
        const float d0p[3] = {dcv.x, dcv.y, dcv.z};
        const int deg = VEC ? 3 : a.D;
        const f3 dir_orig = {mean.x - a.campos[0], mean.y - a.campos[1], mean.z - a.campos[2]};
        const float len = sqrtf(fmaf(dir_orig.z, dir_orig.z, fmaf(dir_orig.y, dir_orig.y, dir_orig.x * dir_orig.x)));
        const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
        // forward colour (same expression as raster_fwd.hip sh_to_rgb) for the clamp mask
        float basis[15];
        int nb = 0;
        float xx = 0, yy = 0, zz = 0, xy = 0, yz = 0, xz = 0;
        if (deg > 0) {
            basis[0] = -SH_C1 * y; basis[1] = SH_C1 * z; basis[2] = -SH_C1 * x; nb = 3;
            if (deg > 1) {
                xx = x * x; yy = y * y; zz = z * z; xy = x * y; yz = y * z; xz = x * z;
                basis[3] = SH_C2[0] * xy;
                basis[4] = SH_C2[1] * yz;
                basis[5] = SH_C2[2] * (2.0f * zz - xx - yy);
                basis[6] = SH_C2[3] * xz;
                basis[7] = SH_C2[4] * (xx - yy);
                nb = 8;
                if (deg > 2) {
                    basis[8] = SH_C3[0] * y * (3.0f * xx - yy);
                    basis[9] = SH_C3[1] * xy * z;
                    basis[10] = SH_C3[2] * y * (4.0f * zz - xx - yy);
                    basis[11] = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                    basis[12] = SH_C3[4] * x * (4.0f * zz - xx - yy);
                    basis[13] = SH_C3[5] * z * (xx - yy);
                    basis[14] = SH_C3[6] * x * (xx - 3.0f * yy);
                    nb = 15;
                }
            }
        }
        float dRGB[3];
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            float r = SH_C0 * d0p[ch];
#pragma unroll
            for (int k = 0; k < 15; k++)
                if (k < nb) r = fmaf(basis[k], SHV(k, ch), r);
            r += 0.5f;
            dRGB[ch] = (r < 0) ? 0.0f : acc[6 + ch];
        }
        st3(a.ddc + 3 * idx, SH_C0 * dRGB[0], SH_C0 * dRGB[1], SH_C0 * dRGB[2]);
        float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
        if (deg > 0) {
            for (int ch = 0; ch < 3; ch++) {
                dx[ch] = -SH_C1 * SHV(2, ch); dy[ch] = -SH_C1 * SHV(0, ch); dz[ch] = SH_C1 * SHV(1, ch);
            }
            if (deg > 1) {
                for (int ch = 0; ch < 3; ch++) {
                    dx[ch] += SH_C2[0] * y * SHV(3, ch) + SH_C2[2] * 2.f * -x * SHV(5, ch) + SH_C2[3] * z * SHV(6, ch) + SH_C2[4] * 2.f * x * SHV(7, ch);
                    dy[ch] += SH_C2[0] * x * SHV(3, ch) + SH_C2[1] * z * SHV(4, ch) + SH_C2[2] * 2.f * -y * SHV(5, ch) + SH_C2[4] * 2.f * -y * SHV(7, ch);
                    dz[ch] += SH_C2[1] * y * SHV(4, ch) + SH_C2[2] * 2.f * 2.f * z * SHV(5, ch) + SH_C2[3] * x * SHV(6, ch);
                }
                if (deg > 2) {
                    for (int ch = 0; ch < 3; ch++) {
                        dx[ch] += (SH_C3[0] * SHV(8, ch) * 3.f * 2.f * xy + SH_C3[1] * SHV(9, ch) * yz + SH_C3[2] * SHV(10, ch) * -2.f * xy +
                                   SH_C3[3] * SHV(11, ch) * -3.f * 2.f * xz + SH_C3[4] * SHV(12, ch) * (-3.f * xx + 4.f * zz - yy) +
                                   SH_C3[5] * SHV(13, ch) * 2.f * xz + SH_C3[6] * SHV(14, ch) * 3.f * (xx - yy));
                        dy[ch] += (SH_C3[0] * SHV(8, ch) * 3.f * (xx - yy) + SH_C3[1] * SHV(9, ch) * xz +
                                   SH_C3[2] * SHV(10, ch) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * SHV(11, ch) * -3.f * 2.f * yz +
                                   SH_C3[4] * SHV(12, ch) * -2.f * xy + SH_C3[5] * SHV(13, ch) * -2.f * yz + SH_C3[6] * SHV(14, ch) * -3.f * 2.f * xy);
                        dz[ch] += (SH_C3[1] * SHV(9, ch) * xy + SH_C3[2] * SHV(10, ch) * 4.f * 2.f * yz +
                                   SH_C3[3] * SHV(11, ch) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * SHV(12, ch) * 4.f * 2.f * xz +
                                   SH_C3[5] * SHV(13, ch) * (xx - yy));
                    }
                }
            }
        }
        // dL/dsh of the active rows (the rest stays zero); VEC: 11 dwordx4 stores + 1 instead of 45 dword stores
        if (VEC) {
            float o[45];
#pragma unroll
            for (int k = 0; k < 15; k++)
#pragma unroll
                for (int ch = 0; ch < 3; ch++) o[3 * k + ch] = basis[k] * dRGB[ch];
#pragma unroll
            for (int i = 0; i < 11; i++)
                *reinterpret_cast<f4u*>(dsh_row + 4 * i) = f4u{o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]};
            dsh_row[44] = o[44];
        } else {
            for (int k = 0; k < nb; k++)
                for (int ch = 0; ch < 3; ch++) dsh_row[3 * k + ch] = basis[k] * dRGB[ch];
        }
        const f3 ddir = {dx[0] * dRGB[0] + dx[1] * dRGB[1] + dx[2] * dRGB[2], dy[0] * dRGB[0] + dy[1] * dRGB[1] + dy[2] * dRGB[2],
                         dz[0] * dRGB[0] + dz[1] * dRGB[1] + dz[2] * dRGB[2]};
        // dnormvdv (auxiliary.h:118-128)
        const f3 v = dir_orig;
        const float sum2 = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
        const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
        dmean.x += ((sum2 - v.x * v.x) * ddir.x - v.y * v.x * ddir.y - v.z * v.x * ddir.z) * invsum32;
        dmean.y += (-v.x * v.y * ddir.x + (sum2 - v.y * v.y) * ddir.y - v.z * v.y * ddir.z) * invsum32;
        dmean.z += (-v.x * v.z * ddir.x - v.y * v.z * ddir.y + (sum2 - v.z * v.z) * ddir.z) * invsum32;
    }
}

// One contributing Gaussian: every gradient output of it (dL/dsh row included) is written here.
__device__ __forceinline__ void gauss_bwd_one(const GaussBwdArgs& a, int idx, const float (&sums)[10]) {
    const int M = a.M;
    float* dsh_row = a.dsh ? a.dsh + (size_t)idx * M * 3 : nullptr;
    // every per-Gaussian input is loaded up front: one HBM round trip instead of dependent ones
    const float4 sp0 = a.sp[2 * (size_t)idx], sp1 = a.sp[2 * (size_t)idx + 1];
    const f3 mean = ld3(a.means3D + 3 * idx);
    f3 scl = {0.f, 0.f, 0.f};
    f4 rot = {0.f, 0.f, 0.f, 0.f};
    if (a.scales) {
        scl = ld3(a.scales + 3 * idx);
        const f4u q = *reinterpret_cast<const f4u*>(a.rotations + 4 * idx);
        rot = {q.x, q.y, q.z, q.w};
    }
    const float opac = a.antialiasing ? a.opacities[idx] : 0.f;
    f3 dcv = {0.f, 0.f, 0.f};
    if (a.sh) dcv = ld3(a.dc + 3 * idx);
    // degree 3, 15 rest rows: the SH row in registers, loaded here with the other inputs (11 dwordx4 + 1)
    const bool shvec = a.sh && a.D >= 3 && M == 15;
    float shv[45];
    if (shvec) {
        const float* shp = a.sh + (size_t)idx * 45;
#pragma unroll
        for (int i = 0; i < 11; i++) {
            const f4u v = *reinterpret_cast<const f4u*>(shp + 4 * i);
            shv[4 * i] = v.x; shv[4 * i + 1] = v.y; shv[4 * i + 2] = v.z; shv[4 * i + 3] = v.w;
        }
        shv[44] = shp[44];
    }
    // a Gaussian with instances was rendered (radii > 0); tested after the input loads are issued, not before them
    if (a.radii[idx] <= 0) return;
    // ---- records -> dL/d(mean2D, conic, opacity, color, invdepth): summed by the wave (see below)
    float acc[10];
#pragma unroll
    for (int v = 0; v < 10; v++) acc[v] = sums[v];
    // moments -> dL/dmean2D, dL/dconic (see render_bwd_tile); o = the AA-scaled opacity of the forward
    {
        const float4 c4 = make_float4(sp0.z, sp0.w, sp1.x, sp1.y);
        const float SGx = acc[0], SGy = acc[1], SGxx = acc[2], SGxy = acc[3], SGyy = acc[4];
        const float so = c4.w;
        acc[0] = -(0.5f * a.W) * (so * fmaf(c4.x, SGx, c4.y * SGy));
        acc[1] = -(0.5f * a.H) * (so * fmaf(c4.z, SGy, c4.y * SGx));
        acc[2] = (-0.5f * so) * SGxx;
        acc[3] = (-0.5f * so) * SGxy;
        acc[4] = (-0.5f * so) * SGyy;
    }
    st3(a.dmeans2D + 3 * idx, acc[0], acc[1], 0.f);
    st3(a.dcolors + 3 * idx, acc[6], acc[7], acc[8]);
    float dLo = acc[5];
    const float dL_dinvd = acc[9];

    // ---- computeCov2DCUDA (backward.cu:149-326)
    // both sources land in registers (a pointer to either would put the local copy on the stack)
    float cbuf[6];
    if (a.cov3D_precomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) cbuf[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        cov3d_fwd(scl, a.scale_mod, rot, cbuf);
    }
    const float* cov3D = cbuf;
    const float h_x = a.focal_x, h_y = a.focal_y;
    Cov2DState st;
    const f3 cv = cov2d_fwd(mean, h_x, h_y, a.tanfovx, a.tanfovy, cov3D, a.view, &st);
    float c_xx = cv.x, c_xy = cv.y, c_yy = cv.z;
    const float h_var = 0.3f;
    float d_inside_root = 0.f;
    if (a.antialiasing) {
        const float det_cov = fmaf(c_xx, c_yy, -(c_xy * c_xy));
        c_xx += h_var; c_yy += h_var;
        const float det_plus = fmaf(c_xx, c_yy, -(c_xy * c_xy));
        const float hs = sqrtf(fmaxf(0.000025f, det_cov / det_plus));
        const float dhs = dLo * opac;
        dLo = dLo * hs;
        d_inside_root = (det_cov / det_plus) <= 0.000025f ? 0.f : dhs / (2 * hs);
    } else {
        c_xx += h_var; c_yy += h_var;
    }
    a.dopacity[idx] = dLo;
    float dcxx = 0.f, dcxy = 0.f, dcyy = 0.f;
    if (a.antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float denom_f = d_inside_root / sq(w * w + w * (x + y) + x * y - z * z);
        dcxx = w * (w * y + y * y + z * z) * denom_f;
        dcyy = w * (w * x + x * x + z * z) * denom_f;
        dcxy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float gcx = acc[2], gcy = acc[3], gcz = acc[4];  // dL/dconic (x, y, w)
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const m3& T = st.T;
    const float T00 = T.m[0][0], T01 = T.m[0][1], T02 = T.m[0][2], T10 = T.m[1][0], T11 = T.m[1][1], T12 = T.m[1][2];
    float dcov[6];
    if (denom2inv != 0) {
        dcxx += denom2inv * (-c_yy * c_yy * gcx + 2 * c_xy * c_yy * gcy + (denom - c_xx * c_yy) * gcz);
        dcyy += denom2inv * (-c_xx * c_xx * gcz + 2 * c_xx * c_xy * gcy + (denom - c_xx * c_yy) * gcx);
        dcxy += denom2inv * 2 * (c_xy * c_yy * gcx - (denom + 2 * c_xy * c_xy) * gcy + c_xx * c_xy * gcz);
        dcov[0] = (T00 * T00 * dcxx + T00 * T10 * dcxy + T10 * T10 * dcyy);
        dcov[3] = (T01 * T01 * dcxx + T01 * T11 * dcxy + T11 * T11 * dcyy);
        dcov[5] = (T02 * T02 * dcxx + T02 * T12 * dcxy + T12 * T12 * dcyy);
        dcov[1] = 2 * T00 * T01 * dcxx + (T00 * T11 + T01 * T10) * dcxy + 2 * T10 * T11 * dcyy;
        dcov[2] = 2 * T00 * T02 * dcxx + (T00 * T12 + T02 * T10) * dcxy + 2 * T10 * T12 * dcyy;
        dcov[4] = 2 * T02 * T01 * dcxx + (T01 * T12 + T02 * T11) * dcxy + 2 * T11 * T12 * dcyy;
    } else {
        for (int i = 0; i < 6; i++) dcov[i] = 0.f;
    }
    *reinterpret_cast<f2u*>(a.dcov3D + 6 * idx) = f2u{dcov[0], dcov[1]};  // 8-B aligned rows: three dwordx2
    *reinterpret_cast<f2u*>(a.dcov3D + 6 * idx + 2) = f2u{dcov[2], dcov[3]};
    *reinterpret_cast<f2u*>(a.dcov3D + 6 * idx + 4) = f2u{dcov[4], dcov[5]};
    const m3& V = st.V;
    const float dT00 = 2 * (T00 * V.m[0][0] + T01 * V.m[0][1] + T02 * V.m[0][2]) * dcxx + (T10 * V.m[0][0] + T11 * V.m[0][1] + T12 * V.m[0][2]) * dcxy;
    const float dT01 = 2 * (T00 * V.m[1][0] + T01 * V.m[1][1] + T02 * V.m[1][2]) * dcxx + (T10 * V.m[1][0] + T11 * V.m[1][1] + T12 * V.m[1][2]) * dcxy;
    const float dT02 = 2 * (T00 * V.m[2][0] + T01 * V.m[2][1] + T02 * V.m[2][2]) * dcxx + (T10 * V.m[2][0] + T11 * V.m[2][1] + T12 * V.m[2][2]) * dcxy;
    const float dT10 = 2 * (T10 * V.m[0][0] + T11 * V.m[0][1] + T12 * V.m[0][2]) * dcyy + (T00 * V.m[0][0] + T01 * V.m[0][1] + T02 * V.m[0][2]) * dcxy;
    const float dT11 = 2 * (T10 * V.m[1][0] + T11 * V.m[1][1] + T12 * V.m[1][2]) * dcyy + (T00 * V.m[1][0] + T01 * V.m[1][1] + T02 * V.m[1][2]) * dcxy;
    const float dT12 = 2 * (T10 * V.m[2][0] + T11 * V.m[2][1] + T12 * V.m[2][2]) * dcyy + (T00 * V.m[2][0] + T01 * V.m[2][1] + T02 * V.m[2][2]) * dcxy;
    const m3& W = st.W;
    const float dJ00 = W.m[0][0] * dT00 + W.m[0][1] * dT01 + W.m[0][2] * dT02;
    const float dJ02 = W.m[2][0] * dT00 + W.m[2][1] * dT01 + W.m[2][2] * dT02;
    const float dJ11 = W.m[1][0] * dT10 + W.m[1][1] * dT11 + W.m[1][2] * dT12;
    const float dJ12 = W.m[2][0] * dT10 + W.m[2][1] * dT11 + W.m[2][2] * dT12;
    const f3 t = st.t;
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = st.xgm * -h_x * tz2 * dJ02;
    const float dty = st.ygm * -h_y * tz2 * dJ12;
    const float dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t.x) * tz3 * dJ02 + (2 * h_y * t.y) * tz3 * dJ12 -
                      dL_dinvd * tz2;
    f3 dmean = tv4x3T({dtx, dty, dtz}, a.view);

    // ---- preprocessCUDA backward: mean2D projection (backward.cu:425-442)
    {
        const float* proj = a.proj;
        const f4 mh = tp4x4(mean, proj);
        const float m_w = 1.0f / (mh.w + 0.0000001f);
        const float mul1 = (proj[0] * mean.x + proj[4] * mean.y + proj[8] * mean.z + proj[12]) * m_w * m_w;
        const float mul2 = (proj[1] * mean.x + proj[5] * mean.y + proj[9] * mean.z + proj[13]) * m_w * m_w;
        const float gx = acc[0], gy = acc[1];
        dmean.x += (proj[0] * m_w - proj[3] * mul1) * gx + (proj[1] * m_w - proj[3] * mul2) * gy;
        dmean.y += (proj[4] * m_w - proj[7] * mul1) * gx + (proj[5] * m_w - proj[7] * mul2) * gy;
        dmean.z += (proj[8] * m_w - proj[11] * mul1) * gx + (proj[9] * m_w - proj[11] * mul2) * gy;
    }

    // ---- computeColorFromSH backward
    if (shvec) {
        sh_bwd<true>(a, idx, mean, dcv, acc, [&](int k, int ch) { return shv[3 * k + ch]; }, dsh_row, dmean);
    } else if (a.sh) {
        const float* __restrict__ sh = a.sh + (size_t)idx * M * 3;
        sh_bwd<false>(a, idx, mean, dcv, acc, [&](int k, int ch) { return sh[3 * k + ch]; }, dsh_row, dmean);
    } else {
        for (int ch = 0; ch < 3; ch++) a.ddc[3 * idx + ch] = 0.f;
    }
    st3(a.dmeans3D + 3 * idx, dmean.x, dmean.y, dmean.z);

    // ---- computeCov3D backward (backward.cu:330-393)
    if (a.scales) {
        const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
        const m3 R = quat_to_R(r, x, y, z);
        const f3 s = {a.scale_mod * scl.x, a.scale_mod * scl.y, a.scale_mod * scl.z};
        m3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
        S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
        const m3 Mm = m3_mul(S, R);
        const m3 dSig = m3_cols(dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                                0.5f * dcov[2], 0.5f * dcov[4], dcov[5]);
        m3 dM = m3_mul(Mm, dSig);
        for (int i = 0; i < 3; i++) for (int jx = 0; jx < 3; jx++) dM.m[i][jx] *= 2.0f;
        const m3 Rt = m3_T(R);
        m3 D = m3_T(dM);
        float dsc[3];
        for (int k = 0; k < 3; k++) dsc[k] = fmaf(Rt.m[k][2], D.m[k][2], fmaf(Rt.m[k][1], D.m[k][1], Rt.m[k][0] * D.m[k][0]));
        st3(a.dscales + 3 * idx, dsc[0], dsc[1], dsc[2]);
        for (int jx = 0; jx < 3; jx++) { D.m[0][jx] *= s.x; D.m[1][jx] *= s.y; D.m[2][jx] *= s.z; }
        float dq[4];
        dq[0] = 2 * z * (D.m[0][1] - D.m[1][0]) + 2 * y * (D.m[2][0] - D.m[0][2]) + 2 * x * (D.m[1][2] - D.m[2][1]);
        dq[1] = 2 * y * (D.m[1][0] + D.m[0][1]) + 2 * z * (D.m[2][0] + D.m[0][2]) + 2 * r * (D.m[1][2] - D.m[2][1]) - 4 * x * (D.m[2][2] + D.m[1][1]);
        dq[2] = 2 * x * (D.m[1][0] + D.m[0][1]) + 2 * r * (D.m[2][0] - D.m[0][2]) + 2 * z * (D.m[1][2] + D.m[2][1]) - 4 * y * (D.m[2][2] + D.m[0][0]);
        dq[3] = 2 * r * (D.m[0][1] - D.m[1][0]) + 2 * x * (D.m[2][0] + D.m[0][2]) + 2 * y * (D.m[1][2] + D.m[2][1]) - 4 * z * (D.m[1][1] + D.m[0][0]);
        *reinterpret_cast<f4u*>(a.drot + 4 * idx) = f4u{dq[0], dq[1], dq[2], dq[3]};
    } else {
        for (int k = 0; k < 3; k++) a.dscales[3 * idx + k] = 0.f;
        for (int k = 0; k < 4; k++) a.drot[4 * idx + k] = 0.f;
    }
}

#ifdef DG_BWD_STATS
__global__ void k_bwd_stats_dump() {
    unsigned long long t[3] = {0, 0, 0};
    for (int b = 0; b < 256; b++)
        for (int i = 0; i < 3; i++) { t[i] += g_bs[b * 4 + i]; g_bs[b * 4 + i] = 0ull; }
    printf("BWDSTATS iterations %llu any_ok %llu ok_pixels %llu util_of_iter %.4f util_of_anyok %.4f\n", t[0], t[1], t[2],
           t[0] ? (double)t[2] / (256.0 * (double)t[0]) : 0.0, t[1] ? (double)t[2] / (256.0 * (double)t[1]) : 0.0);
}
#endif
void launch_render_bwd(const RenderBwdArgs& a, uint32_t* counters, hipStream_t s, bool order_ready) {
    (void)counters;
    if (a.num_tiles <= 0) return;
    if (a.order && !order_ready) k_bwd_order<<<1, 1024, 0, s>>>(a);
    k_render_bwd<<<(a.num_tiles + 3) / 4, 256, 0, s>>>(a);
#ifdef DG_BWD_STATS
    k_bwd_stats_dump<<<1, 1, 0, s>>>();
#endif
}
void launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    // sized for the phase-1 capacity (E1 <= K1); phase-2 chunks are picked up by the grid-stride loops
    const uint32_t chunks = (a.K1 + SUM_CHUNK - 1) / SUM_CHUNK;
    const uint32_t sum_blocks = chunks ? (chunks + 3) / 4 : 1u;
    const uint32_t aux_blocks = ((uint32_t)a.P + AUX_SPAN - 1) / AUX_SPAN;
    k_gauss_sum<<<sum_blocks + aux_blocks, 256, 0, s>>>(a, sum_blocks);
    const uint32_t live_blocks = chunks ? (chunks + LIVE_CHUNKS - 1) / LIVE_CHUNKS : 1u;
    k_gauss_live<<<live_blocks, LIVE_THREADS, 0, s>>>(a);
}

}  // namespace gs

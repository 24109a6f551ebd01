// wave_sort.h -- per-tile depth sort of an instance list by one wave64 (in registers + wave-private LDS), shared by
// k_tile_dsort (sortscan.hip) and the phase-1 render, which sorts its own tile before compositing it
// (raster_fwd.hip).  See sortscan.hip "binning by tile" for the design.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sortscan.h"

namespace gs {

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// inclusive prefix sum over the wave64 by DPP (row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15/31
// across rows): six VALU adds, no LDS
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// lanes of this wave (among active ones) whose 8-bit digit equals mine
__device__ __forceinline__ uint64_t peer_mask(uint32_t digit, bool active) {
    uint64_t m = __ballot(active);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const bool bit = (digit >> b) & 1u;
        const uint64_t bal = __ballot(bit && active);
        m &= bit ? bal : ~bal;
    }
    return active ? m : 0ull;
}

constexpr int DS_WAVE_MAX = 512;           // per-wave capacity inside the render (8 items per lane)
constexpr int DS_ROWS = DS_WAVE_MAX / 64;
constexpr int DS_WAVE_MAX2 = 1024;         // per-wave capacity of the standalone sort kernels (16 per lane)
constexpr int DS_ROWS2 = DS_WAVE_MAX2 / 64;

__device__ __forceinline__ uint32_t ds_key(const DSortArgs& a, uint32_t v) {
    return a.ikey[v < a.n_inst ? v : a.n_inst - 1];
}
__device__ __forceinline__ uint32_t ds_gid(const DSortArgs& a, uint32_t v) {
    return a.eg[v < a.n_inst ? v : a.n_inst - 1];
}

// wave min / max by the DPP scan's pattern (identity from rows and lanes without a source); lane 63 holds the result
template <bool MAX>
__device__ __forceinline__ uint32_t wave_minmax_u32(uint32_t x) {
    constexpr int ID = MAX ? 0 : -1;
    auto f = [](uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(ID, (int)x, 0x111, 0xf, 0xf, false));
    x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(ID, (int)x, 0x112, 0xf, 0xf, false));
    x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(ID, (int)x, 0x114, 0xf, 0xf, false));
    x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(ID, (int)x, 0x118, 0xf, 0xf, false));
    x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(ID, (int)x, 0x142, 0xa, 0xf, false));
    x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(ID, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) { return wave_minmax_u32<false>(x); }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) { return wave_minmax_u32<true>(x); }
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63);
}
__device__ __forceinline__ int passes_for(uint32_t range) { return range ? (32 - __clz((int)range) + 7) >> 3 : 0; }

// Stable in-wave LSD radix sort of (k, v) over the R = ceil(n/64) register rows, digits of k below 8*passes.
// Items i >= n must carry k = 0xffffffff (they stay last).
template <int ROWS>
__device__ __forceinline__ void wave_radix(uint32_t (&k)[ROWS], uint32_t (&v)[ROWS], int R, int passes,
                                           uint32_t* cnt, uint32_t* lk, uint32_t* lv, int lane) {
    uint32_t rank[ROWS];
    const uint64_t lt = lanemask_lt();
    for (int p = 0; p < passes; p++) {
        const int shift = 8 * p;
#pragma unroll
        for (int q = 0; q < 4; q++) cnt[q * 64 + lane] = 0u;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            if (r < R) {
                const uint32_t d = (k[r] >> shift) & 0xffu;
                const uint64_t m = peer_mask(d, true);
                const uint32_t before = (uint32_t)__popcll(m & lt);
                const uint32_t cur = cnt[d];
                rank[r] = cur + before;
                if (before == 0) cnt[d] = cur + (uint32_t)__popcll(m);  // LDS ops of one wave complete in order
            }
        }
        __builtin_amdgcn_wave_barrier();
        {  // exclusive scan of the 256 digit counts, 4 per lane
            const uint32_t c0 = cnt[4 * lane], c1 = cnt[4 * lane + 1], c2 = cnt[4 * lane + 2], c3 = cnt[4 * lane + 3];
            const uint32_t loc = c0 + c1 + c2 + c3;
            const uint32_t x = wave_incl_scan(loc);
            const uint32_t ex = x - loc;
            __builtin_amdgcn_wave_barrier();
            cnt[4 * lane] = ex; cnt[4 * lane + 1] = ex + c0; cnt[4 * lane + 2] = ex + c0 + c1;
            cnt[4 * lane + 3] = ex + c0 + c1 + c2;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            if (r < R) {
                const uint32_t pos = cnt[(k[r] >> shift) & 0xffu] + rank[r];
                lk[pos] = k[r];
                lv[pos] = v[r];
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            if (r < R) { k[r] = lk[r * 64 + lane]; v[r] = lv[r * 64 + lane]; }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Relative sort keys of the wave's items (key(v) - min over the list; 0xffffffff padding); returns the range.
template <int ROWS, typename KeyFn>
__device__ __forceinline__ uint32_t wave_rel_keys(uint32_t (&k)[ROWS], const uint32_t (&v)[ROWS], int R, int n,
                                                  int lane, KeyFn&& key) {
    uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const int i = r * 64 + lane;
        k[r] = (r < R && i < n) ? key(v[r]) : 0u;
    }
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const int i = r * 64 + lane;
        if (r < R && i < n) {
            kmin = k[r] < kmin ? k[r] : kmin;
            kmax = k[r] > kmax ? k[r] : kmax;
        }
    }
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const int i = r * 64 + lane;
        k[r] = (i < n) ? k[r] - kmin : 0xffffffffu;
    }
    return kmax - kmin;
}

// Sort tile `tile`'s list (min_n < n <= 64 ROWS) into (depth key, Gaussian index) order and write it back to s_e
// (and, when ids_out is given, to ids_out[0..n), e.g. wave-private LDS).  cnt [256], lk/lv [64 ROWS]: wave-private
// LDS scratch.  Returns n; a list outside (min_n, 64 ROWS] is left alone (the caller handles it).
template <int ROWS>
__device__ __forceinline__ int wave_sort_tile(const DSortArgs& a, int tile, int lane, uint32_t* cnt, uint32_t* lk,
                                              uint32_t* lv, uint32_t* ids_out, int min_n = 1) {
    const uint2 rg = a.ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= min_n || n <= 1 || n > 64 * ROWS) return n;
    uint32_t* se = a.s_e + rg.x;
    const int R = (n + 63) >> 6;
    uint32_t k[ROWS], v[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const int i = r * 64 + lane;
        v[r] = (r < R && i < n) ? se[i] : 0u;
    }
    const uint32_t range = wave_rel_keys(k, v, R, n, lane, [&](uint32_t x) { return ds_key(a, x); });
#ifndef DG_DSORT_NOSORT
    wave_radix<ROWS>(k, v, R, passes_for(range), cnt, lk, lv, lane);
#endif
    // Equal depth keys (i >= n carry 0xffffffff and never match a real relative key) must end up in Gaussian
    // index order; the counting sort left them in arrival order.  They sit next to each other after the sort, so
    // odd-even transposition between equal-key neighbours fixes them (one round per element of the longest run).
    bool tie = false;
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        if (r < R) {
            uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k[r], 0x138, 0xf, 0xf, false);  // wave_shr:1
            if (lane == 0) prev = r > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)k[r > 0 ? r - 1 : 0], 63) : ~k[r];
            const int i = r * 64 + lane;
            tie |= (i < n) && prev == k[r];
        }
    }
    if (__any(tie)) {
        uint32_t gid[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const int i = r * 64 + lane;
            gid[r] = (r < R && i < n) ? ds_gid(a, v[r]) : 0xffffffffu;
        }
        for (int round = 0; round < 64 * ROWS; round++) {
            bool changed = false;
#pragma unroll
            for (int par = 0; par < 2; par++) {
                uint32_t nv[ROWS], ng[ROWS];
#pragma unroll
                for (int r = 0; r < ROWS; r++) {
                    nv[r] = v[r]; ng[r] = gid[r];
                    if (r >= R) continue;
                    const int i = r * 64 + lane;
                    // right neighbour (i + 1) and left neighbour (i - 1)
                    uint32_t kr = __shfl_down(k[r], 1), vr = __shfl_down(v[r], 1), gr = __shfl_down(gid[r], 1);
                    uint32_t kl = __shfl_up(k[r], 1), vl = __shfl_up(v[r], 1), gl = __shfl_up(gid[r], 1);
                    if (r + 1 < ROWS) {
                        const int rn = r + 1 < ROWS ? r + 1 : r;
                        const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)k[rn], 0);
                        const uint32_t v0 = (uint32_t)__builtin_amdgcn_readlane((int)v[rn], 0);
                        const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)gid[rn], 0);
                        if (lane == 63) { kr = k0; vr = v0; gr = g0; }
                    }
                    if (r > 0) {
                        const int rp = r > 0 ? r - 1 : 0;
                        const uint32_t k63 = (uint32_t)__builtin_amdgcn_readlane((int)k[rp], 63);
                        const uint32_t v63 = (uint32_t)__builtin_amdgcn_readlane((int)v[rp], 63);
                        const uint32_t g63 = (uint32_t)__builtin_amdgcn_readlane((int)gid[rp], 63);
                        if (lane == 0) { kl = k63; vl = v63; gl = g63; }
                    }
                    if (i < n) {
                        if ((i & 1) == par) {  // left element of the pair (i, i + 1)
                            if (i + 1 < n && kr == k[r] && gr < gid[r]) { nv[r] = vr; ng[r] = gr; changed = true; }
                        } else if (i > 0) {    // right element of the pair (i - 1, i)
                            if (kl == k[r] && gid[r] < gl) { nv[r] = vl; ng[r] = gl; changed = true; }
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < ROWS; r++) { v[r] = nv[r]; gid[r] = ng[r]; }
            }
            if (!__any(changed)) break;
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
        const int i = r * 64 + lane;
        if (r < R && i < n) {
            se[i] = v[r];
            if (ids_out) ids_out[i] = v[r];
        }
    }
    __builtin_amdgcn_wave_barrier();
    return n;
}

// ---- long lists (n > a wave's capacity): one 256-thread block, LSD radix through global scratch (k_a, k_b, s_tmp)
constexpr int BS_RADIX = 256;
constexpr int BS_WAVES = 4;

// One stable LSD step of the long-list sort by a 256-thread team: (key(v) - kmin) digits, (keys, vals) ping-pong
// through global scratch in 256-item chunks.  `key` maps a value to its sort key.  Result in va.  The team is threads
// 0..255 of the block; a larger block's other threads only take part in the barriers (k_render_fwd2x's 1024).
template <typename KeyFn>
__device__ __forceinline__ void block_radix_global(uint32_t*& va, uint32_t*& vb, uint32_t* ka, uint32_t* kb, uint32_t n,
                                   KeyFn&& key, uint32_t* s_base, uint32_t (*s_wh)[BS_RADIX], uint32_t (*s_red)[BS_WAVES]) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const bool on = t < 256;
    const uint64_t lt = lanemask_lt();
    uint32_t kmin = 0xffffffffu, kmax = 0u;
    for (uint32_t i = t; on && i < n; i += 256) {
        const uint32_t kk = key(va[i]);
        ka[i] = kk;
        kmin = kk < kmin ? kk : kmin;
        kmax = kk > kmax ? kk : kmax;
    }
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
    __syncthreads();
    if (on && lane == 0) { s_red[0][w] = kmin; s_red[1][w] = kmax; }
    __syncthreads();
    kmin = s_red[0][0]; kmax = s_red[1][0];
    for (int q = 1; q < BS_WAVES; q++) {
        kmin = s_red[0][q] < kmin ? s_red[0][q] : kmin;
        kmax = s_red[1][q] > kmax ? s_red[1][q] : kmax;
    }
    const int passes = passes_for(kmax - kmin);
    for (int p = 0; p < passes; p++) {
        const int shift = 8 * p;
        __syncthreads();
        if (on) s_base[t] = 0u;
        __syncthreads();
        for (uint32_t i = t; on && i < n; i += 256) atomicAdd(&s_base[((ka[i] - kmin) >> shift) & 0xffu], 1u);
        __syncthreads();
        {  // exclusive scan of the digit counts (thread t = digit t)
            const uint32_t c = on ? s_base[t] : 0u;
            const uint32_t x = wave_incl_scan(c);
            if (on && lane == 63) s_red[0][w] = x;
            __syncthreads();
            uint32_t off = 0;
            for (int q = 0; q < w && q < BS_WAVES; q++) off += s_red[0][q];
            if (on) s_base[t] = off + x - c;
        }
        __syncthreads();
        for (uint32_t c0 = 0; c0 < n; c0 += 256) {
            const uint32_t i = c0 + t;
            const bool act = on && i < n;
            const uint32_t kk = act ? ka[i] : 0u;
            const uint32_t val = act ? va[i] : 0u;
            const uint32_t d = ((kk - kmin) >> shift) & 0xffu;
            const uint64_t m = peer_mask(d, act);
            const uint32_t before = (uint32_t)__popcll(m & lt);
            if (on) {
#pragma unroll
                for (int q = 0; q < BS_WAVES; q++) s_wh[q][t] = 0u;
            }
            __syncthreads();
            if (act && before == 0) s_wh[w][d] = (uint32_t)__popcll(m);
            __syncthreads();
            if (act) {
                uint32_t pos = s_base[d] + before;
                for (int q = 0; q < w; q++) pos += s_wh[q][d];
                kb[pos] = kk;
                vb[pos] = val;
            }
            __syncthreads();
            if (on) s_base[t] += s_wh[0][t] + s_wh[1][t] + s_wh[2][t] + s_wh[3][t];
            __syncthreads();
        }
        uint32_t* tk = ka; ka = kb; kb = tk;
        uint32_t* tv = va; va = vb; vb = tv;
    }
    __syncthreads();
}

// Block-level sort of one long list (n > DS_WAVE_MAX): LSD radix through global scratch; with equal keys it sorts by
// Gaussian index first and then, stably, by key.  Threads 0..255 work; any others only join the barriers.
__device__ __forceinline__ void block_sort_long(const DSortArgs& a, int tile, uint32_t* s_base, uint32_t (*s_wh)[BS_RADIX],
                                uint32_t (*s_red)[BS_WAVES], int* s_tie) {
    const int t = threadIdx.x;
    const bool on = t < 256;
    const uint2 rg = a.ranges[tile];
    const uint32_t n = rg.y - rg.x;
    uint32_t *va = a.s_e + rg.x, *vb = a.s_tmp + rg.x;
    auto dkey = [&](uint32_t x) { return ds_key(a, x); };
    block_radix_global(va, vb, a.k_a + rg.x, a.k_b + rg.x, n, dkey, s_base, s_wh, s_red);
    if (t == 0) *s_tie = 0;
    __syncthreads();
    for (uint32_t i = t + 1; on && i < n; i += 256)
        if (ds_key(a, va[i]) == ds_key(a, va[i - 1])) *s_tie = 1;
    __syncthreads();
    if (*s_tie) {  // rare: order by Gaussian index first, then stably by key
        block_radix_global(va, vb, a.k_a + rg.x, a.k_b + rg.x, n, [&](uint32_t x) { return ds_gid(a, x); }, s_base,
                           s_wh, s_red);
        block_radix_global(va, vb, a.k_a + rg.x, a.k_b + rg.x, n, dkey, s_base, s_wh, s_red);
    }
    if (va != a.s_e + rg.x)  // result in the scratch values: copy back into s_e
        for (uint32_t i = t; on && i < n; i += 256) a.s_e[rg.x + i] = va[i];
    __syncthreads();
}

}  // namespace gs

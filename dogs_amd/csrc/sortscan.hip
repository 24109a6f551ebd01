// sortscan.hip -- device-wide exclusive scan and stable LSD radix sort for gfx950 (wave64).
//
// Radix sort: 8-bit digits, reduce-then-scan per pass:
//   rs_upsweep   one workgroup per 4096-key tile, per-digit counts -> counts[digit][tile]
//   rs_scan      one workgroup per digit, exclusive scan over tiles, digit totals
//   rs_downsweep stable rank inside the tile (wave-level peer masks from 8 ballots, each wave owns a
//                contiguous 1024-key sub-tile so ranking needs no barrier), LDS reorder, coalesced
//                scatter of contiguous digit runs.
// Stability is what makes the (tile, depth, index) order of the reference's cub::SortPairs fall out
// of two cheap sorts (DESIGN.md "Binning").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "sortscan.h"
#include "wave_sort.h"

namespace gs {

constexpr int RS_THREADS = 256;
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_ITEMS = 16;                       // keys per thread
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;     // 4096
constexpr int RS_WAVE_TILE = 64 * RS_ITEMS;        // 1024 contiguous keys per wave
constexpr int RS_RADIX = 256;

// n_dev (optional): element count read on the device, <= the capacity n the grid was sized for; tiles past
// it count nothing and scatter nothing, so a launch sized for a capacity sorts a prefix without a host sync.
__device__ __forceinline__ uint32_t eff_n(uint32_t n, const uint32_t* n_dev) {
    if (!n_dev) return n;
    const uint32_t d = *n_dev;
    return d < n ? d : n;
}

__global__ void __launch_bounds__(RS_THREADS) rs_upsweep(const uint32_t* __restrict__ keys, uint32_t ncap,
                                                         const uint32_t* __restrict__ n_dev, int shift,
                                                         uint32_t* __restrict__ counts, uint32_t ntiles) {
    __shared__ uint32_t hist[RS_RADIX];
    const int t = threadIdx.x;
    hist[t] = 0;
    __syncthreads();
    const uint32_t n = eff_n(ncap, n_dev);
    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * RS_TILE;
    if (n == 0u) return;  // nothing to sort (rs_scan and rs_downsweep leave too)
    if (base >= n) {  // past the device-side count: nothing to count (uniform per block)
        counts[(size_t)t * ntiles + tile] = 0u;
        return;
    }
    const int lane = __lane_id();
#pragma unroll 4
    for (int r = 0; r < RS_ITEMS; r++) {
        const uint32_t i = base + r * RS_THREADS + t;
        const bool act = i < n;
        const uint32_t d = act ? (keys[i] >> shift) & 0xffu : 0u;
        const uint64_t m = peer_mask(d, act);
        if (act && (__ffsll((unsigned long long)m) - 1) == lane) atomicAdd(&hist[d], (uint32_t)__popcll(m));
    }
    __syncthreads();
    counts[(size_t)t * ntiles + tile] = hist[t];
}

// one block per digit: exclusive scan over tiles in place, total -> digit_total[d]
__global__ void __launch_bounds__(1024) rs_scan(uint32_t* __restrict__ counts, uint32_t ntiles,
                                                uint32_t* __restrict__ digit_total,
                                                const uint32_t* __restrict__ n_dev) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (n_dev && *n_dev == 0u) return;  // nothing to sort: every downsweep tile leaves too
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t* row = counts + (size_t)blockIdx.x * ntiles;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t b = 0; b < ntiles; b += 1024) {
        const uint32_t i = b + t;
        const uint32_t v = i < ntiles ? row[i] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        if (w == 0) {
            uint32_t s = lane < 16 ? wsum[lane] : 0u;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const uint32_t y = __shfl_up(s, o);
                if (lane >= o) s += y;
            }
            if (lane < 16) wsum[lane] = s;
        }
        __syncthreads();
        const uint32_t excl = carry + (w ? wsum[w - 1] : 0u) + x - v;
        if (i < ntiles) row[i] = excl;
        __syncthreads();
        if (t == 1023) carry = excl + v;
        __syncthreads();
    }
    if (t == 0) digit_total[blockIdx.x] = carry;
}

__global__ void __launch_bounds__(RS_THREADS) rs_downsweep(const uint32_t* __restrict__ keys_in,
                                                           const uint32_t* __restrict__ vals_in,
                                                           uint32_t* __restrict__ keys_out,
                                                           uint32_t* __restrict__ vals_out, uint32_t ncap,
                                                           const uint32_t* __restrict__ n_dev, int shift,
                                                           const uint32_t* __restrict__ counts, uint32_t ntiles,
                                                           const uint32_t* __restrict__ digit_total) {
    __shared__ uint32_t s_keys[RS_TILE];
    __shared__ uint32_t s_vals[RS_TILE];
    __shared__ uint32_t whist[RS_WAVES][RS_RADIX];
    __shared__ uint32_t s_tile_start[RS_RADIX];  // tile-local start of each digit run
    __shared__ uint32_t s_gbase[RS_RADIX];       // global start of this tile's run of each digit
    __shared__ uint32_t s_wtmp[RS_WAVES];

    const int t = threadIdx.x, lane = __lane_id(), w = t >> 6;
    const uint32_t n = eff_n(ncap, n_dev);
    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * RS_TILE;
    if (base >= n) return;  // whole block (uniform)
#pragma unroll
    for (int k = 0; k < RS_WAVES; k++) whist[k][t] = 0;
    // exclusive scan of digit totals (256) -> global digit base
    {
        const uint32_t v = digit_total[t];
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wtmp[w] = x;
        __syncthreads();
        uint32_t off = 0;
        for (int k = 0; k < w; k++) off += s_wtmp[k];
        s_gbase[t] = off + x - v + counts[(size_t)t * ntiles + tile];
    }
    // per-wave stable ranking over its contiguous 1024-key sub-tile
    uint32_t my_key[RS_ITEMS], my_val[RS_ITEMS], my_rank[RS_ITEMS];
    const uint32_t wbase = base + w * RS_WAVE_TILE;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; r++) {
        const uint32_t i = wbase + r * 64 + lane;
        const bool act = i < n;
        my_key[r] = act ? keys_in[i] : 0xffffffffu;
        my_val[r] = act ? (vals_in ? vals_in[i] : i) : 0u;
    }
#pragma unroll
    for (int r = 0; r < RS_ITEMS; r++) {
        const uint32_t i = wbase + r * 64 + lane;
        const bool act = i < n;
        const uint32_t d = (my_key[r] >> shift) & 0xffu;
        const uint64_t m = peer_mask(d, act);
        const uint32_t before = (uint32_t)__popcll(m & lanemask_lt());
        const uint32_t cur = act ? whist[w][d] : 0u;
        my_rank[r] = cur + before;
        // the group's leader publishes the new count; LDS ops of one wave complete in order
        if (act && before == 0) whist[w][d] = cur + (uint32_t)__popcll(m);
    }
    __syncthreads();
    // per digit: offsets of each wave's run, and the tile-local start of the digit run
    {
        uint32_t run = 0;
        uint32_t woff[RS_WAVES];
#pragma unroll
        for (int k = 0; k < RS_WAVES; k++) { woff[k] = run; run += whist[k][t]; }
        // tile-local exclusive scan over digits of `run`
        uint32_t x = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        __syncthreads();
        if (lane == 63) s_wtmp[w] = x;
        __syncthreads();
        uint32_t off = 0;
        for (int k = 0; k < w; k++) off += s_wtmp[k];
        const uint32_t start = off + x - run;
        s_tile_start[t] = start;
#pragma unroll
        for (int k = 0; k < RS_WAVES; k++) whist[k][t] = start + woff[k];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ITEMS; r++) {
        const uint32_t i = wbase + r * 64 + lane;
        if (i < n) {
            const uint32_t d = (my_key[r] >> shift) & 0xffu;
            const uint32_t lp = whist[w][d] + my_rank[r];
            s_keys[lp] = my_key[r];
            s_vals[lp] = my_val[r];
        }
    }
    __syncthreads();
    const uint32_t cnt = (n - base) < (uint32_t)RS_TILE ? (n - base) : (uint32_t)RS_TILE;
#pragma unroll 4
    for (int r = 0; r < RS_ITEMS; r++) {
        const uint32_t j = r * RS_THREADS + t;
        if (j < cnt) {
            const uint32_t k = s_keys[j];
            const uint32_t d = (k >> shift) & 0xffu;
            const uint32_t o = s_gbase[d] + (j - s_tile_start[d]);
            keys_out[o] = k;
            vals_out[o] = s_vals[j];
        }
    }
}

size_t radix_sort_temp_bytes(uint32_t n) {
    const uint32_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    return ((size_t)RS_RADIX * (ntiles ? ntiles : 1) + RS_RADIX) * sizeof(uint32_t);
}

int radix_sort_pairs(uint32_t* keys0, uint32_t* vals0, uint32_t* keys1, uint32_t* vals1, const uint32_t* vals_first,
                     uint32_t n, int begin_bit, int end_bit, void* temp, hipStream_t stream, const uint32_t* n_dev) {
    if (n == 0) return 0;
    const uint32_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    uint32_t* counts = (uint32_t*)temp;
    uint32_t* totals = counts + (size_t)RS_RADIX * ntiles;
    uint32_t *kin = keys0, *vin = vals0, *kout = keys1, *vout = vals1;
    int pass = 0;
    for (int b = begin_bit; b < end_bit; b += 8, pass++) {
        rs_upsweep<<<ntiles, RS_THREADS, 0, stream>>>(kin, n, n_dev, b, counts, ntiles);
        rs_scan<<<RS_RADIX, 1024, 0, stream>>>(counts, ntiles, totals, n_dev);
        rs_downsweep<<<ntiles, RS_THREADS, 0, stream>>>(kin, pass == 0 ? vals_first : vin, kout, vout, n, n_dev, b,
                                                        counts, ntiles, totals);
        uint32_t* tk = kin; kin = kout; kout = tk;
        uint32_t* tv = vin; vin = vout; vout = tv;
    }
    return pass & 1;  // 1 -> result in keys1/vals1, 0 -> in keys0/vals0
}

// ---------------- exclusive scan (u32) ----------------
constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 8;
constexpr int SC_TILE = SC_THREADS * SC_ITEMS;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t& total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < SC_THREADS / 64; k++) { if (k < w) off += s_w[k]; tot += s_w[k]; }
    __syncthreads();
    total = tot;
    return off + x - v;
}

// element i of the scanned sequence: in[i], or 0 when a mask is given and lt_keys[i] >= *lt_thr
__device__ __forceinline__ uint32_t sc_val(const uint32_t* in, const uint32_t* lt_keys, uint32_t thr, uint32_t i) {
    const uint32_t v = in[i];
    return (lt_keys && !(lt_keys[i] < thr)) ? 0u : v;
}

__global__ void __launch_bounds__(SC_THREADS) sc_reduce(const uint32_t* __restrict__ in,
                                                        const uint32_t* __restrict__ lt_keys,
                                                        const uint32_t* __restrict__ lt_thr, uint32_t n,
                                                        uint32_t* __restrict__ block_sums,
                                                        const uint32_t* __restrict__ gate) {
    __shared__ uint32_t s_w[SC_THREADS / 64];
    if (gate && *gate == 0u) return;
    const uint32_t thr = lt_keys ? *lt_thr : 0u;
    const uint32_t base = blockIdx.x * SC_TILE + threadIdx.x * SC_ITEMS;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SC_ITEMS; k++) {
        const uint32_t i = base + k;
        if (i < n) s += sc_val(in, lt_keys, thr, i);
    }
    uint32_t tot;
    block_excl_scan(s, s_w, tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SC_THREADS) sc_scan_sums(uint32_t* __restrict__ sums, uint32_t nb,
                                                           uint32_t* __restrict__ total_out,
                                                           const uint32_t* __restrict__ gate) {
    __shared__ uint32_t s_w[SC_THREADS / 64];
    __shared__ uint32_t carry;
    if (gate && *gate == 0u) {
        if (threadIdx.x == 0 && total_out) *total_out = 0u;
        return;
    }
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b = 0; b < nb; b += SC_THREADS) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < nb ? sums[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(v, s_w, tot);
        const uint32_t c = carry;
        if (i < nb) sums[i] = c + ex;
        __syncthreads();
        if (threadIdx.x == 0) carry = c + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ void __launch_bounds__(SC_THREADS) sc_downsweep(const uint32_t* __restrict__ in,
                                                           const uint32_t* __restrict__ lt_keys,
                                                           const uint32_t* __restrict__ lt_thr, uint32_t n,
                                                           const uint32_t* __restrict__ block_sums,
                                                           uint32_t* __restrict__ out,
                                                           const uint32_t* __restrict__ gate) {
    __shared__ uint32_t s_w[SC_THREADS / 64];
    if (gate && *gate == 0u) return;
    const uint32_t thr = lt_keys ? *lt_thr : 0u;
    const uint32_t base = blockIdx.x * SC_TILE + threadIdx.x * SC_ITEMS;
    uint32_t v[SC_ITEMS];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SC_ITEMS; k++) {
        const uint32_t i = base + k;
        v[k] = i < n ? sc_val(in, lt_keys, thr, i) : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t run = block_sums[blockIdx.x] + block_excl_scan(s, s_w, tot);
#pragma unroll
    for (int k = 0; k < SC_ITEMS; k++) {
        const uint32_t i = base + k;
        if (i < n) out[i] = run;
        run += v[k];
    }
}

size_t scan_temp_bytes(uint32_t n) {
    const uint32_t nb = (n + SC_TILE - 1) / SC_TILE;
    return (size_t)(nb ? nb : 1) * sizeof(uint32_t);
}

void exclusive_scan(const uint32_t* in, uint32_t n, uint32_t* out, uint32_t* total, void* temp, hipStream_t stream,
                    const uint32_t* gate, const uint32_t* lt_keys, const uint32_t* lt_thr) {
    const uint32_t nb = (n + SC_TILE - 1) / SC_TILE;
    uint32_t* sums = (uint32_t*)temp;
    if (n == 0) {
        (void)hipMemsetAsync(total, 0, sizeof(uint32_t), stream);
        return;
    }
    sc_reduce<<<nb, SC_THREADS, 0, stream>>>(in, lt_keys, lt_thr, n, sums, gate);
    sc_scan_sums<<<1, SC_THREADS, 0, stream>>>(sums, nb, total, gate);
    sc_downsweep<<<nb, SC_THREADS, 0, stream>>>(in, lt_keys, lt_thr, n, sums, out, gate);
}


// ---------------- binning by tile: counting sort + exact per-tile order ----------------
// The instances of a phase are binned by tile with a counting sort: the binning walk counts per tile (atomics),
// k_tile_offsets turns the counts into ranges, and the emission walk places each instance at an atomic arrival
// slot of its tile (raster_fwd.hip k_bin_emit).  The order inside a tile is then whatever the atomics produced;
// k_tile_dsort puts every tile's list into the reference's exact (depth bits, Gaussian index) order -- a total
// order, so the result does not depend on the atomics.
//   k_tile_dsort       one wave per tile, lists up to DS_WAVE_MAX: items in registers (8 per lane), LSD radix
//                      over the tile's key range (keys relative to the tile minimum, 8-bit digits, only as many
//                      passes as the range needs), wave-level peer-mask ranking, LDS scatter.  Runs of equal
//                      depth keys are put in Gaussian index order by odd-even transposition between neighbours.
//   k_tile_dsort_long  longer lists (queued by k_tile_dsort): one block per tile, LSD radix through global scratch
//                      in 256-item chunks; with equal keys it sorts by Gaussian index first and then, stably, by key.
__global__ void __launch_bounds__(1024) k_tile_offsets(uint32_t* __restrict__ tile_cnt, uint32_t num_tiles,
                                                       uint2* __restrict__ ranges, const uint32_t* __restrict__ gate) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    if (gate && *gate == 0u) return;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_carry = 0u;
    __syncthreads();
    for (uint32_t b = 0; b < num_tiles; b += 1024) {
        const uint32_t i = b + t;
        const uint32_t v = i < num_tiles ? tile_cnt[i] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t off = s_carry, tot = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) { if (k < w) off += s_w[k]; tot += s_w[k]; }
        const uint32_t ex = off + x - v;
        if (i < num_tiles) { ranges[i] = make_uint2(ex, ex + v); tile_cnt[i] = ex; }
        __syncthreads();
        if (t == 0) s_carry += tot;
        __syncthreads();
    }
}

void tile_offsets(uint32_t* tile_cnt, uint32_t num_tiles, uint2* ranges, hipStream_t stream, const uint32_t* gate) {
    if (num_tiles) k_tile_offsets<<<1, 1024, 0, stream>>>(tile_cnt, num_tiles, ranges, gate);
}

#ifndef DG_BO_OLD
// Block 0: exclusive scan of the wave totals in place (+ total); block 1: the per-tile ranges (tile_offsets).
// 16 contiguous items per thread (four 16-B loads), so one round covers 16 * NT items -- a 1e6-Gaussian view's 15625
// wave totals in one round at NT = 1024: one HBM round trip, one barrier.  The wave scan is DPP (row_shr 1/2/4/8,
// row_bcast 15/31; no LDS), the wave sums meet in LDS.
#ifndef DG_BO_ITEMS
#define DG_BO_ITEMS 16
#endif
constexpr int BO_ITEMS = DG_BO_ITEMS;
template <int NT>
__global__ void __launch_bounds__(NT) k_bin_offsets(uint32_t* __restrict__ wtot, uint32_t n,
                                                      uint32_t* __restrict__ total, uint32_t* __restrict__ tile_cnt,
                                                      uint32_t num_tiles, uint2* __restrict__ ranges,
                                                      const uint32_t* __restrict__ gate) {
    constexpr int NW = NT / 64;
    constexpr uint32_t PER = (uint32_t)BO_ITEMS * NT;
    __shared__ uint32_t s_w[2][NW];
    const bool tiles = blockIdx.x == 1;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // the gate is tested after the first round's loads are issued (in bounds either way: the arrays are sized for n),
    // so the block waits on one round trip, not two
    const uint32_t gv = gate ? *gate : 1u;
    const uint32_t N = tiles ? num_tiles : n;
    uint32_t* src = tiles ? tile_cnt : wtot;
    // the 16-B paths need 16-B aligned arrays (the carver's are 256-B aligned); otherwise element by element
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | (tiles ? reinterpret_cast<uintptr_t>(ranges) : 0u)) & 15u) == 0u;
    auto load = [&](uint32_t b, uint32_t (&v)[BO_ITEMS]) {
        const uint32_t i0 = b + (uint32_t)BO_ITEMS * (uint32_t)t;
        if (vec && i0 + BO_ITEMS <= N) {
            const uint4* s4 = reinterpret_cast<const uint4*>(src + i0);
#pragma unroll
            for (int q = 0; q < BO_ITEMS / 4; q++) {
                const uint4 u = s4[q];
                v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < BO_ITEMS; k++) v[k] = i0 + k < N ? src[i0 + k] : 0u;
        }
    };
    uint32_t carry = 0u;
    int par = 0;
    // the next round's loads are issued before this round's scan (its in-place stores cover other items), so a
    // multi-round scan (5e6 Gaussians: 78k wave totals, 5 rounds) waits on memory once, not once per round
    uint32_t nv[BO_ITEMS];
    if (N) load(0u, nv);
    for (uint32_t b = 0; b < N; b += PER, par ^= 1) {
        const uint32_t i0 = b + (uint32_t)BO_ITEMS * (uint32_t)t;
        uint32_t v[BO_ITEMS];
#pragma unroll
        for (int k = 0; k < BO_ITEMS; k++) v[k] = nv[k];
        if (b + PER < N) load(b + PER, nv);  // block-uniform
        if (gv == 0u) break;  // block-uniform: nothing to scan (total = carry = 0)
        uint32_t loc = 0u;
#pragma unroll
        for (int k = 0; k < BO_ITEMS; k++) loc += v[k];
        const uint32_t x = wave_incl_scan(loc);
        if (lane == 63) s_w[par][w] = x;
        __syncthreads();  // s_w[par] complete; the other parity's readers finished before the previous round's barrier
        uint32_t off = carry, tot = 0u;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t s = s_w[par][k];
            off += k < w ? s : 0u;
            tot += s;
        }
        carry += tot;
        uint32_t ex = off + x - loc;
        if (vec && i0 + BO_ITEMS <= N) {
            if (tiles) {
#pragma unroll
                for (int k = 0; k < BO_ITEMS; k += 2) {
                    const uint32_t e1 = ex + v[k], e2 = e1 + v[k + 1];
                    reinterpret_cast<uint4*>(ranges + i0)[k / 2] = make_uint4(ex, e1, e1, e2);
                    ex = e2;
                }
                ex = off + x - loc;
            }
            uint32_t o[BO_ITEMS];
#pragma unroll
            for (int k = 0; k < BO_ITEMS; k++) { o[k] = ex; ex += v[k]; }
            uint4* d4 = reinterpret_cast<uint4*>(src + i0);
#pragma unroll
            for (int q = 0; q < BO_ITEMS / 4; q++) d4[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < BO_ITEMS; k++) {
                if (i0 + k < N) {
                    if (tiles) ranges[i0 + k] = make_uint2(ex, ex + v[k]);
                    src[i0 + k] = ex;
                }
                ex += v[k];
            }
        }
    }
    if (!tiles && t == 0) *total = carry;
}
#else
// Block 0: exclusive scan of the wave totals in place (+ total); block 1: the per-tile ranges (tile_offsets).
// 4 items per thread per 4096-item round, wave shuffle scan + 16 wave sums in LDS, running carry.  The loads of
// BO_ROUNDS rounds are issued before the first scan (one HBM round trip per 16384 items instead of one per round:
// a 1e6-Gaussian view has 15625 wave totals, so the whole scan waits on memory once).
constexpr int BO_ROUNDS = 4;
template <int NT>
__global__ void __launch_bounds__(NT) k_bin_offsets(uint32_t* __restrict__ wtot, uint32_t n,
                                                      uint32_t* __restrict__ total, uint32_t* __restrict__ tile_cnt,
                                                      uint32_t num_tiles, uint2* __restrict__ ranges,
                                                      const uint32_t* __restrict__ gate) {
    constexpr int NW = NT / 64;
    __shared__ uint32_t s_w[NW];
    __shared__ uint32_t s_carry;
    const bool tiles = blockIdx.x == 1;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (gate && *gate == 0u) {
        if (!tiles && t == 0) *total = 0u;
        return;
    }
    const uint32_t N = tiles ? num_tiles : n;
    uint32_t* src = tiles ? tile_cnt : wtot;
    if (t == 0) s_carry = 0u;
    __syncthreads();
    for (uint32_t sb = 0; sb < N; sb += (4u * NT) * BO_ROUNDS) {
      uint32_t pv[BO_ROUNDS][4];
#pragma unroll
      for (int r = 0; r < BO_ROUNDS; r++) {
          const uint32_t i0 = sb + (4u * NT) * r + 4u * (uint32_t)t;
#pragma unroll
          for (int k = 0; k < 4; k++) pv[r][k] = i0 + k < N ? src[i0 + k] : 0u;
      }
#pragma unroll
      for (int r = 0; r < BO_ROUNDS; r++) {
        const uint32_t b = sb + (4u * NT) * r;
        if (b >= N) break;  // block-uniform
        const uint32_t i0 = b + 4u * (uint32_t)t;
        const uint32_t* v = pv[r];
        const uint32_t loc = v[0] + v[1] + v[2] + v[3];
        uint32_t x = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t off = s_carry, tot = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) { if (k < w) off += s_w[k]; tot += s_w[k]; }
        uint32_t ex = off + x - loc;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (i0 + k < N) {
                if (tiles) { ranges[i0 + k] = make_uint2(ex, ex + v[k]); tile_cnt[i0 + k] = ex; }
                else wtot[i0 + k] = ex;
            }
            ex += v[k];
        }
        __syncthreads();
        if (t == 0) s_carry += tot;
        __syncthreads();
      }
    }
    if (!tiles && t == 0) *total = s_carry;
}
#endif

void bin_offsets(uint32_t* wtot, uint32_t n, uint32_t* total, uint32_t* tile_cnt, uint32_t num_tiles, uint2* ranges,
                 hipStream_t stream, const uint32_t* gate, bool small_blocks) {
    // small_blocks: 256-thread blocks (more rounds), which find room beside another stream's kernel (the native step's
    // overlapped update kept a 1024-thread block of this launch waiting until it ended)
    if (small_blocks) k_bin_offsets<256><<<2, 256, 0, stream>>>(wtot, n, total, tile_cnt, num_tiles, ranges, gate);
    else k_bin_offsets<1024><<<2, 1024, 0, stream>>>(wtot, n, total, tile_cnt, num_tiles, ranges, gate);
}

// One wave per tile, lists up to DS_WAVE_MAX2 (16 items per lane); min_n: only lists longer than that (the phase-1
// render sorts the shorter ones itself).  Longer lists are queued for k_tile_dsort_long.
template <int MIN_N>
__global__ void __launch_bounds__(256) k_tile_dsort(DSortArgs a) {
    __shared__ uint32_t s_cnt[4][RS_RADIX];
    __shared__ uint32_t s_k[4][DS_WAVE_MAX2];
    __shared__ uint32_t s_v[4][DS_WAVE_MAX2];
    if (a.gate && *a.gate == 0u) return;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + w;
    if (tile >= a.num_tiles) return;
    if (a.only && !a.only[tile]) return;
    const int n = wave_sort_tile<DS_ROWS2>(a, tile, lane, s_cnt[w], s_k[w], s_v[w], nullptr, MIN_N);
    if (n > DS_WAVE_MAX2 && lane == 0) a.long_list[atomicAdd(a.long_cnt, 1u)] = (uint32_t)tile;
}

// Long lists: one block per queued tile.  Grid-stride over the queue; its length is device-side (no host sync).
__global__ void __launch_bounds__(256) k_tile_dsort_long(DSortArgs a) {
    __shared__ uint32_t s_base[BS_RADIX];
    __shared__ uint32_t s_wh[BS_WAVES][BS_RADIX];
    __shared__ uint32_t s_red[2][BS_WAVES];
    __shared__ int s_tie;
    if (a.gate && *a.gate == 0u) return;
    const uint32_t nl = *a.long_cnt;
    for (uint32_t li = blockIdx.x; li < nl; li += gridDim.x)
        block_sort_long(a, (int)a.long_list[li], s_base, s_wh, s_red, &s_tie);
}

// The lists longer than the render's fused sort (n > DS_WAVE_MAX) in ONE launch of few blocks: block b scans the
// ranges of tiles [64 b, 64 b + 64) (16 per wave), each wave sorts the lists it finds up to DS_WAVE_MAX2 itself
// and queues longer ones in the block's LDS; after a barrier the block sorts its queue (block_sort_long).  A 1080p
// view has a handful of such lists, so this replaces a 2040-block launch that mostly exits plus a 256-block
// grid-stride launch: the same two sort routines, so the same order.
constexpr int DSM_TILES = 64;
#ifndef DG_DSORT_DENSE_SPLIT
#define DG_DSORT_DENSE_SPLIT 1
#endif
constexpr bool DSORT_DENSE_SPLIT = DG_DSORT_DENSE_SPLIT;
// tiles per block (4 = one per wave .. DSM_TILES): the host picks 4 when the phase-1 capacity per tile makes most lists
// longer than the render's wave capacity (5e6 Gaussians at 1080p: ~1500 rect units per tile), where 16 sorts in a row
// per wave over 128 blocks took ~500 us per view against ~125 with a wave per tile
__global__ void __launch_bounds__(256) k_tile_dsort_merged(DSortArgs a, int tpb) {
    __shared__ uint32_t s_cnt[4][RS_RADIX];
    __shared__ uint32_t s_k[4][DS_WAVE_MAX2];
    __shared__ uint32_t s_v[4][DS_WAVE_MAX2];
    __shared__ uint32_t s_q[DSM_TILES];
    __shared__ uint32_t s_nq;
    __shared__ int s_tie;
    // the gate is read with the tile lengths below (in bounds either way), one memory round trip instead of two
    const uint32_t gv = a.gate ? *a.gate : 1u;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) s_nq = 0u;
    __syncthreads();
    const int t0 = blockIdx.x * tpb + w * (tpb / 4);
    // the wave's tile lengths in one load round (lane i: tile t0 + i), then only the lists past the render's own sort
    // capacity are visited -- at 1e6 Gaussians almost none, and the 16 dependent range loads of a tile-by-tile walk
    // were the whole launch (~6 us)
    for (int i0 = 0; i0 < tpb / 4; i0 += 64) {
        const int tile = t0 + i0 + lane;
        bool longer = false;
        if (i0 + lane < tpb / 4 && tile < a.num_tiles) {
            const uint2 rg = a.ranges[tile];
            longer = rg.y - rg.x > (uint32_t)DS_WAVE_MAX;
        }
        uint64_t m = gv ? __ballot(longer) : 0ull;
        while (m) {
            const int i = i0 + (int)__builtin_ctzll(m);
            m &= m - 1;
            const int n = wave_sort_tile<DS_ROWS2>(a, t0 + i, lane, s_cnt[w], s_k[w], s_v[w], nullptr, DS_WAVE_MAX);
            if (n > DS_WAVE_MAX2 && lane == 0) s_q[atomicAdd(&s_nq, 1u)] = (uint32_t)(t0 + i);
        }
    }
    __syncthreads();
    const uint32_t nq = s_nq;  // 0 when gated
    uint32_t* scr = &s_k[0][0];  // the wave sorts are done: their scratch serves the block sort
    for (uint32_t q = 0; q < nq; q++)
        block_sort_long(a, (int)s_q[q], scr, reinterpret_cast<uint32_t(*)[BS_RADIX]>(scr + BS_RADIX),
                        reinterpret_cast<uint32_t(*)[BS_WAVES]>(scr + BS_RADIX * (1 + BS_WAVES)), &s_tie);
}

void tile_depth_sort_long_only(const DSortArgs& a, hipStream_t stream) {
    if (a.num_tiles <= 0) return;
#ifdef DG_DSORT_TWO_LAUNCHES
    k_tile_dsort<DS_WAVE_MAX><<<(a.num_tiles + 3) / 4, 256, 0, stream>>>(a);
    k_tile_dsort_long<<<256, 256, 0, stream>>>(a);
#else
    // dense lists (rect units per tile past 1.5x the wave capacity; ~0.57 precise instances per rect unit): a wave per
    // tile, and the lists past a wave's reach queued for a grid of block sorts -- many of them at 5e6 Gaussians, where
    // a block's own queue (up to four lists in a row) left the launch waiting on its slowest blocks
    const bool dense = (uint64_t)a.n_inst > (uint64_t)a.num_tiles * (uint64_t)(DS_WAVE_MAX * 3 / 2);
    if (dense && DSORT_DENSE_SPLIT) {
        k_tile_dsort<DS_WAVE_MAX><<<(a.num_tiles + 3) / 4, 256, 0, stream>>>(a);
        k_tile_dsort_long<<<1024, 256, 0, stream>>>(a);
        return;
    }
    const int tpb = dense ? 4 : DSM_TILES;
    k_tile_dsort_merged<<<(a.num_tiles + tpb - 1) / tpb, 256, 0, stream>>>(a, tpb);
#endif
}

void tile_depth_sort(const DSortArgs& a, hipStream_t stream) {
    if (a.num_tiles <= 0) return;
    k_tile_dsort<1><<<(a.num_tiles + 3) / 4, 256, 0, stream>>>(a);
    k_tile_dsort_long<<<256, 256, 0, stream>>>(a);
}

}  // namespace gs

// sortscan.h -- host entry points of the device-wide scan / radix sort (sortscan.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gs {

// the multi-block replay order of the phase-2 launches (gs_common.h order_hist_piece / order_scatter_piece)
constexpr int ORDER_NB = 256, ORDER_TILES = 256;
__host__ __device__ constexpr int order_blocks(int num_tiles) { return (num_tiles + ORDER_TILES - 1) / ORDER_TILES; }

// Stable LSD radix sort of (key, value) pairs over bits [begin_bit, end_bit), 8 bits per pass.
// Pass 0 reads values from vals_first (nullptr -> value = input index).  Ping-pongs between the
// (keys0, vals0) and (keys1, vals1) buffers; keys0 holds the input.  Returns 1 when the result is in
// keys1/vals1, 0 when it is in keys0/vals0.  n sizes the launch; when n_dev is given the kernels sort
// only the first min(*n_dev, n) elements (device-side count, no host sync).
size_t radix_sort_temp_bytes(uint32_t n);
int radix_sort_pairs(uint32_t* keys0, uint32_t* vals0, uint32_t* keys1, uint32_t* vals1, const uint32_t* vals_first,
                     uint32_t n, int begin_bit, int end_bit, void* temp, hipStream_t stream,
                     const uint32_t* n_dev = nullptr);

// out[i] = sum_{j<i} v[j], v[j] = in[j] (or 0 when lt_keys is given and lt_keys[j] >= *lt_thr, a device-side
// threshold);  *total = full sum (device pointer).
// gate (optional, device): when *gate == 0 nothing is read or written except *total = 0.
size_t scan_temp_bytes(uint32_t n);
void exclusive_scan(const uint32_t* in, uint32_t n, uint32_t* out, uint32_t* total, void* temp, hipStream_t stream,
                    const uint32_t* gate = nullptr, const uint32_t* lt_keys = nullptr, const uint32_t* lt_thr = nullptr);

// ranges[t] = [start, end) from the per-tile counts (exclusive scan, one block), and tile_cnt set to start so that it
// serves as the per-tile arrival cursor (an atomic increment returns the instance's slot, no ranges load).  gate (optional, device): nothing when *gate == 0.
void tile_offsets(uint32_t* tile_cnt, uint32_t num_tiles, uint2* ranges, hipStream_t stream,
                  const uint32_t* gate = nullptr);

// Both scans of a binning phase in one launch of two single-block scans: wtot[0..n) -> exclusive prefix in place
// (*total = sum) and tile_offsets() above.  For n <= BIN_OFFSETS_MAX_N (longer wave-total arrays take
// exclusive_scan + tile_offsets).  gate as above (*total = 0 when gated).
#ifndef DG_BIN_OFFSETS_MAX_N
#define DG_BIN_OFFSETS_MAX_N 262144
#endif
constexpr uint32_t BIN_OFFSETS_MAX_N = DG_BIN_OFFSETS_MAX_N;
void bin_offsets(uint32_t* wtot, uint32_t n, uint32_t* total, uint32_t* tile_cnt, uint32_t num_tiles, uint2* ranges,
                 hipStream_t stream, const uint32_t* gate = nullptr, bool small_blocks = false);

// Per-tile sort of instance lists into (depth key, Gaussian index) order (sortscan.hip k_tile_dsort):
// s_e[ranges[t].x .. ranges[t].y) is reordered in place by (ikey[v], eg[v]), whatever its input order.
struct DSortArgs {
    int num_tiles;
    const uint2* ranges;
    uint32_t* s_e;              // tile-binned instance list (values are instance indices)
    uint32_t* s_tmp;            // scratch values, same indexing as s_e (long lists)
    uint32_t *k_a, *k_b;        // scratch keys, same indexing as s_e (long lists)
    const uint32_t* ikey;       // instance -> 32-bit depth key of its Gaussian
    const uint32_t* eg;         // instance -> Gaussian index (tie order)
    uint32_t n_inst;            // bound of ikey / eg
    const uint8_t* only;        // optional: sort only tiles t with only[t] != 0
    const uint32_t* gate;       // optional (device): nothing when *gate == 0
    uint32_t* long_list;        // [num_tiles] queue of tiles longer than the per-wave capacity
    uint32_t* long_cnt;         // device queue length, zeroed beforehand
};
void tile_depth_sort(const DSortArgs& a, hipStream_t stream);
// Only the lists longer than the render's per-wave capacity (DS_WAVE_MAX): a wave per list up to DS_WAVE_MAX2, a block
// per longer one; the phase-1 render sorts the others itself (wave_sort.h).
void tile_depth_sort_long_only(const DSortArgs& a, hipStream_t stream);
}  // namespace gs

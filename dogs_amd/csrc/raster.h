// raster.h -- kernel argument blocks and launchers of the gfx950 rasterizer (raster_fwd.hip, raster_bwd.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sortscan.h"

namespace gs {

// Splat record: everything binning and compositing read per Gaussian, in ONE 32-B record so a
// depth-ordered or instance-ordered gather touches one cache line instead of one per array.
//   sp[2g]     = {mean2D.x, mean2D.y, conic.a, conic.b}
//   sp[2g + 1] = {conic.c, opacity * AA scale, bits(x0 | x1 << 16), bits(y0 | y1 << 16)}   (tile rect)
__device__ __forceinline__ void sp_rect(const float4& s1, int& x0, int& y0, int& x1, int& y1) {
    const uint32_t rx = __float_as_uint(s1.z), ry = __float_as_uint(s1.w);
    x0 = (int)(rx & 0xffffu); x1 = (int)(rx >> 16); y0 = (int)(ry & 0xffffu); y1 = (int)(ry >> 16);
}

struct PreArgs {
    int P, D, M, W, H, tiles_x, tiles_y;
    int antialiasing, prefiltered;
    float tanfovx, tanfovy, focal_x, focal_y, scale_mod;
    const float *means3D, *scales, *rotations, *opacities, *dc, *sh, *colors, *cov3D_precomp;
    const float *view, *proj, *campos;
    int* radii;
    float4* sp;         // splat record, 2 x float4 per Gaussian (see SP_* below)
    uint32_t* depthkey; // float bits of view z, 0xffffffff when culled (empty tile rect)
    uint32_t* hist;     // [DH_BINS] depth histogram, zeroed here
    uint32_t* cnt;      // tile-rect area (0 when culled)
    uint32_t* rcnt;     // records per Gaussian, zeroed here (written by the emission kernels)
    unsigned long long* rect_part;  // [blocks] per-block sums of rect areas (k_depth_cut totals them: num_rendered);
                                    // bit 63 = a prefiltered violation in the block (-> counters[CNT_ERR])
    uint32_t* err;
    unsigned long long* unf_rows;  // [unf_words] per-tile-row bitmasks of unfinished tiles, zeroed here (set by the render)
    int unf_words;
    // optional (the native training step): the parameter activations of GaussianSplatModel done here -- opacity =
    // sigmoid(raw_o), scaling = exp(raw_s), rotation = normalize(raw_q) written to opacities / scales / rotations
    // (which then are outputs) for every Gaussian -- and part_sc[block] = the block's sum of prod(scaling, 1)
    const float *raw_o, *raw_s, *raw_q;
    float* part_sc;
    uint64_t* zero_stamp;  // with raw_*: *zero_stamp = stamp when some activated scaling is exactly 0
    uint64_t stamp;
};

// Counters block at the head of the geometry state (device, uint32 slots).
enum {
    CNT_K = 0,          // total tile-rect area of the visible Gaussians (bounds the instance count)
    CNT_ERR = 1,        // prefiltered violation
    CNT_RECT_LO = 2,    // num_rendered (sum of rect areas), u64 in slots 2..3
    CNT_THR = 4,        // depth-key threshold: Gaussians with key < thr are binned in phase 1
    CNT_E1 = 5,         // instances of phase 1 (allocated by the emission)
    CNT_UNFINISHED = 6, // tiles with live pixels after phase 1 (only counted when CNT_CUT)
    CNT_K2 = 7,         // phase-2 instances
    CNT_CUT = 8,        // E1 < K: the phase-1 lists are prefixes
    CNT_INVD = 9,       // backward: any(dL/dinvdepth != 0) (zeroed with the block by the forward)
    CNT_LONG = 11,      // phase-1 tiles queued for the long-list depth sort
    CNT_LONG2 = 12,     // phase-2 tiles queued for the long-list depth sort
    CNT_UNF2 = 13,      // unfinished tiles with phase-2 instances (RenderArgs::unf_sorted entries)
    CNT_PREV_UNF = 14,  // unfinished tiles of the previous phase-2 launch at this image size (adaptive capacity)
    CNT_PREV_K2 = 15,   // phase-2 instances of that launch
};

// Depth histogram of the prefix cut: bins of 2^DH_SHIFT key ulps (1/64 of a binade) from the near plane up;
// DH_BINS covers 16 binades (z in [0.2, 13107)), farther keys share the last bin.
constexpr int DH_SHIFT = 17;
constexpr int DH_BINS = 1024;

// Depth-prefix binning (DESIGN.md "Binning"): phase 1 bins only the first E1 <= C1 instances of the global depth
// order, which is a prefix of every tile's list; phase 2 bins the rest only for tiles phase 1 left unfinished.
struct RenderArgs {
    int W, H, tiles_x, num_tiles;
    uint32_t K, P;          // bounds of s_e/eg and of the geometry arrays
    const uint2* ranges;
    const uint32_t* s_e;   // sorted instance -> emission index
    const uint32_t* eg;    // emission index -> Gaussian
    // phase 2 (resume) / phase-1 bookkeeping
    int phase;                  // 1 or 2
    const uint2* ranges1;       // phase 2: the phase-1 ranges (contributor numbering continues after them)
    uint32_t* counters;         // CNT_* (phase 1 reads CNT_CUT, counts CNT_UNFINISHED)
    uint8_t* unfinished;        // [num_tiles]
    uint32_t* unf_list;         // [num_tiles] phase 1 appends each unfinished tile (counters[CNT_UNFINISHED] slots);
                                // phase 2 walks this list with a small grid instead of a block per tile
    float4* resume;             // [H*W] raw colour + live flag of unfinished tiles' pixels
    uint2* ranges2_zero;        // phase 1: phase-2 range of each tile it marks unfinished, reset to empty
    const float4* sp;
    const float4* rgbi;
    const float* bg;
    float *out_color, *out_invd, *final_T, *img_color, *img_invd;
    uint32_t *n_contrib, *max_contrib;
    uint32_t* gcount;           // optional (count mode): contributing pixels per Gaussian, accumulated
    // phase 1: each wave first sorts its tile's list (<= DS_WAVE_MAX; longer ones were sorted beforehand by
    // tile_depth_sort_long_only) into the reference order, writes it back for the backward and composites it from
    // wave-private LDS -- the latency-bound sort overlaps the VALU-bound compositing of other waves
    int fuse_sort;
    DSortArgs ds;
    uint32_t* probe;            // optional (phase 2, adaptive capacity): [1] <- counters[CNT_K2]
    unsigned long long* unf_rows;  // phase 1: bit tx % 64 of word ty * unf_rw + tx / 64 set for each unfinished tile
    int unf_rw;
    uint32_t* order;            // phase 2 (k_render_fwd2, optional): out, the backward's replay order (front blocks)
    uint32_t* ohist;            // phase 2 with order: the replay-order bucket counts / cursors (order_scatter_piece)
    const uint32_t* unf_sorted; // phase 2 (optional): the unfinished tiles with phase-2 instances, longest list first
                                // (counters[CNT_UNF2] entries; k_bin_emit<2>'s sort block), walked instead of unf_list
    // phase 1 (optional): block 0 copies hc_src[0..16) to hc_dst[0..16), a coherent pinned host buffer, then sets
    // hc_dst[16] = hc_seq; the host spins on that word (the forward's early counter read without a copy launch or an
    // event; the PCIe round trip hides inside the render)
    const uint32_t* hc_src;
    uint32_t* hc_dst;
    uint32_t hc_seq;
};

struct RenderBwdArgs {
    int W, H, tiles_x, num_tiles;
    uint32_t K, K1, P;       // capacities: per-instance state (global index), phase-1 binning, Gaussians
    const uint2* ranges;
    const uint32_t* max_contrib;
    const uint32_t* s_e;
    const uint32_t* eg;
    const uint2* ranges2;       // phase-2 lists (nullptr when phase 2 did not run)
    const uint32_t* s_e2;       // sorted phase-2 instance -> local emission index
    const uint32_t* eg2;        // local phase-2 emission index -> Gaussian
    const uint32_t* counters;   // CNT_E1: global emission index of phase-2 local index 0
    const uint8_t* unfinished;  // ranges2[t] is valid only where unfinished[t]
    const float4* sp;
    const float4* rgbi;
    const float* bg;
    const float *final_T, *img_color, *img_invd;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    const float* dL_dinvd;   // may be null
    float* rec;              // [K][REC_STRIDE] per-instance gradient record
    uint8_t* flag;           // [K1] record written, phase-1 instances (binning block; zeroed by the emission)
    uint8_t* flag2;          // phase-2 instances (binning2 block), local index: flag2[e - E1]; null without phase 2
    uint32_t* order;         // [num_tiles] scratch: tiles in descending replay length (launch order)
    float* zero_base;        // optional: [zero_count] floats zero-filled by the replay waves (gradient outputs)
    size_t zero_count;
};

struct GaussBwdArgs {
    int P, D, M, W, H, antialiasing;
    uint32_t K;
    float tanfovx, tanfovy, focal_x, focal_y, scale_mod;
    const float *means3D, *scales, *rotations, *opacities, *dc, *sh, *cov3D_precomp;
    const float *view, *proj, *campos;
    const int* radii;
    const uint32_t* dkey;    // forward depth keys (bits of the view z)
    const float4* sp;        // splat records (conic + AA-scaled opacity)
    float* rec;              // per-instance records; k_gauss_sum overwrites a contributing Gaussian's last one
    const uint8_t* flag;     // record written: phase 1 (binning block)
    const uint8_t* flag2;    // phase 2, local index (binning2 block)
    float *dmeans2D, *dcolors, *dopacity, *dmeans3D, *dcov3D, *ddc, *dsh, *dscales, *drot, *depth;
    int outputs_zeroed;      // the nine gradient outputs were zero-filled by k_render_bwd
    // k_gauss_sum walks the instance slots [0, E1 + K2) in chunks of SUM_CHUNK; owner of slot e: eg[e] (phase 1,
    // e < E1) or eg2[e - E1] (phase 2)
    const uint32_t* eg;
    const uint32_t* eg2;     // null: no phase-2 block
    const uint32_t* counters;  // CNT_E1, CNT_K2
    uint32_t K1;             // phase-1 capacity (the forward's num_instances token)
    // k_gauss_sum -> k_gauss_live: per chunk, the contributing Gaussians as (last instance slot, Gaussian index)
    // (live_list[chunk * SUM_CHUNK + j], j < live_cnt[chunk]); their record sums overwrite that slot's record.  The
    // index rides along so that k_gauss_live loads the sums and every per-Gaussian input in one round trip (no owner
    // lookup between them)
    uint2* live_list;        // [chunks * SUM_CHUNK]
    uint32_t* live_cnt;      // [chunks]
};
// floats per instance record: the 10 moments of backward.cu's per-splat terms (40 B; the sum pass overwrites a
// contributing Gaussian's last record with its 10 sums, the owner comes from eg / eg2).  48-B records (the 10 moments +
// the owner, float4-aligned) cost the replay's stores and the sum pass's loads 20% more bytes.
#ifndef DG_REC_STRIDE
#define DG_REC_STRIDE 10
#endif
constexpr int REC_STRIDE = DG_REC_STRIDE;
static_assert(REC_STRIDE == 10 || REC_STRIDE == 12, "DG_REC_STRIDE: 10 or 12");
#ifndef DG_SUM_STEPS
#define DG_SUM_STEPS 2
#endif
constexpr uint32_t SUM_STEPS = DG_SUM_STEPS;      // 64-instance steps per record-sum chunk
constexpr uint32_t SUM_CHUNK = 64u * SUM_STEPS;

void launch_preprocess(const PreArgs& a, hipStream_t s);
// hist[DH_BINS] (zeroed by the preprocess) += precise counts by depth bin
void launch_depth_hist(int P, const uint32_t* dkey, const uint32_t* cnt, uint32_t* hist, hipStream_t s);
// counters[K, THR, E1, CUT] from the histogram (phase-1 capacity cap); resets the per-view counters and zeroes
// the per-tile counters of both binning phases (tile_cnt, tile_cnt2 [num_tiles]) and the replay-order histogram after
// tile_cnt2 (tile_cnt2 + num_tiles, 2 * ORDER_NB words)
// It also totals the preprocess's per-block rect-area sums into counters[CNT_RECT_LO..+1] (num_rendered) and their
// error bits into counters[CNT_ERR] (one atomic per block on a single address costs ~10 us per 1e6 Gaussians:
// cross-XCD serialization), and writes every other counter slot, so the block needs no memset per view.  probe
// (optional, device, per image size): moved into counters[CNT_PREV_UNF] and cleared.
void launch_depth_cut(const uint32_t* hist, uint32_t cap, uint32_t* counters, uint32_t* tile_cnt, uint32_t* tile_cnt2,
                      uint32_t num_tiles, const unsigned long long* rect_part, uint32_t nparts, uint32_t* probe,
                      hipStream_t s);
// launch_depth_hist + launch_depth_cut
void launch_depth_hist_cut(int P, const uint32_t* dkey, const uint32_t* cnt, uint32_t* hist, uint32_t cap,
                           uint32_t* counters, uint32_t* tile_cnt, uint32_t* tile_cnt2, uint32_t num_tiles,
                           const unsigned long long* rect_part, uint32_t nparts, uint32_t* probe, hipStream_t s);
// Binning walk of one phase (phase 1: Gaussians with key < counters[CNT_THR]; phase 2: those past it, only instances
// in tiles phase 1 left unfinished): k_bin_count (precise cull walk -> rcnt, per-wave totals, per-tile counts),
// exclusive scan of the wave totals (*total = the phase's instance count), per-tile ranges, k_bin_emit (first_e;
// eg/ikey per instance; instances grouped by tile in s_e, in arrival order until tile_depth_sort).
// Phase-2 kernels are gated on counters[CNT_UNFINISHED] (device): no-ops when phase 1 finished every tile.
struct BinArgs {
    int P, tiles_x, num_tiles;
    const uint32_t* dkey;
    const float4* sp;
    const uint32_t* counters;    // CNT_THR, CNT_E1 (phase 2), CNT_UNFINISHED
    const uint8_t* unf;          // phase 2: unfinished tiles
    const uint32_t* sat;         // phase 2: summed-area table of unf
    uint32_t* wtot;              // [bin_waves(P)] per-wave totals, scanned in place
    uint64_t* wmask;             // [bin_waves(P)] per-wave member ballot of the count pass, read by the emission
                                 // (fat waves: the member count)
    uint32_t* mlist;             // [P] fat waves: wave w's members (offsets from its first Gaussian), count pass
    uint32_t cap;                // capacity of the instance arrays
    uint32_t *first_e, *rcnt;
    uint32_t *eg, *ikey;         // per instance: Gaussian, depth key
    uint8_t* flag;               // per instance: the backward's record-written flag, zeroed here
    // colour of the binned Gaussians (computeColorFromSH), written by k_bin_emit -- or, colors_later (phase 1, the
    // native step's overlapped SH update), by launch_binned_colors after the emission
    int colors_later;
    int D, M;
    const float *means3D, *campos, *dc, *sh, *colors;
    float4* rgbi;
    uint32_t* tile_cnt;          // [num_tiles] zero on entry: counts, then arrival cursors (from the range starts)
    uint2* ranges;               // [num_tiles] per-tile [start, end) of s_e
    uint32_t* s_e;               // instances grouped by tile
    const unsigned long long* unf_rows;  // phase 2: per-row bitmasks of the unfinished tiles (RenderArgs::unf_rows)
    int unf_rw;                  // words per tile row
    int unf_th;                  // tile rows
    uint32_t* probe;             // optional (phase 2, adaptive capacity): [0] <- counters[CNT_UNFINISHED]
    // optional (phase 2): the emission's front blocks histogram the backward's replay-order buckets into ohist
    // (order_hist_piece; k_render_fwd2 scatters the order): a finished tile's phase-1 max contributor, an unfinished
    // tile's phase-1 + phase-2 list lengths
    uint32_t* ohist;
    const uint32_t* max_contrib;
    const uint2* ranges1;
    // optional (phase 2): one more front block of the emission writes the unfinished tiles that got phase-2 instances,
    // longest list first, to unf_sorted (counters[CNT_UNF2] of them): k_render_fwd2's first-dispatched blocks take the
    // longest tiles, so those do not share a compute unit with another tile's block
    const uint32_t* unf_list;
    uint32_t* unf_sorted;
    // [bin_waves(P) * KM_STEPS] (phase 1): the count pass's kept ballot of each of a wave's first KM_STEPS walk steps;
    // the emission walks the same candidates in the same steps and takes `kept` from here (no per-tile power test)
    uint64_t* kmask;
};
#ifndef DG_KM_STEPS
#define DG_KM_STEPS 8
#endif
constexpr int KM_STEPS = DG_KM_STEPS;  // 0: the emission recomputes every test
void launch_bin(int phase, const BinArgs& a, uint32_t* total, void* scan_tmp, hipStream_t s,
                hipEvent_t wait_before_emit = nullptr);
// rgbi of the phase-1 Gaussians that got instances (rcnt > 0, key < thr), for an emission run with colors_later
void launch_binned_colors(const BinArgs& a, hipStream_t s);
size_t bin_scan_temp_bytes(int P);
int bin_waves(int P);
// probe (optional, device): receives counters[CNT_UNFINISHED] (read back by the next view's k_depth_cut)
void launch_unfinished_sat(const uint32_t* counters, const uint8_t* unfinished, int tiles_x, int tiles_y,
                           uint32_t* sat, hipStream_t s, uint32_t* probe = nullptr);
void launch_render_fwd(const RenderArgs& a, hipStream_t s);
uint32_t preprocess_blocks(int P);  // k_preprocess's grid (PreArgs::part_sc entries)
bool render_fwd2_orders();
bool bin_emit_orders();
// count mode: score[i] = gcount[i] x the (AA-scaled) opacity of splat record i (0 when culled)
void launch_count_score(int P, const int* radii, const float4* sp, const uint32_t* gcount, float* score,
                        hipStream_t s);
void launch_cull_log_threshold(int64_t n, const float* opacity, float* thr, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t s);
void launch_filter(const PreArgs& a, hipStream_t s);
// the replay; order_ready: the forward's phase-2 emission already wrote the replay order, else one block sorts it
void launch_render_bwd(const RenderBwdArgs& a, uint32_t* counters, hipStream_t s, bool order_ready);
void launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t s);

}  // namespace gs

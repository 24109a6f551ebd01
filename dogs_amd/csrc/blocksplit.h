// blocksplit.h -- Grid2D block split kernels (blocksplit.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {
constexpr uint32_t BOX_MAX = 64;  // = DG_MAX_BOXES; the per-point membership is one u64 mask
struct BoxSet {                   // by value as a kernel argument (2.1 KB)
    uint32_t C;
    int has_T;
    double T[6];
    double box[BOX_MAX][4];       // A0 A1 B0 B1
};
struct BoxOffsets {
    uint32_t C;
    uint32_t first[BOX_MAX];      // start of box k's members in the concatenated list
};
uint32_t box_blocks(uint32_t N);
// labels / transformed may be null; masks [N]; cnt [C * box_blocks(N)] (box-major)
void launch_box_test(uint32_t N, const double* pts, uint32_t stride, const BoxSet& bs, uint8_t* labels,
                     double* transformed, uint64_t* masks, uint32_t* cnt, hipStream_t s);
// cnt -> exclusive per-box block offsets in place, total [C]
void launch_box_scan(uint32_t N, uint32_t C, uint32_t* cnt, uint32_t* total, hipStream_t s);
void launch_box_scatter(uint32_t N, const uint64_t* masks, const uint32_t* cnt, const BoxOffsets& off,
                        uint32_t* members, hipStream_t s);
}  // namespace gs

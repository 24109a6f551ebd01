// blocksplit.hip -- Grid2D block split of a scene's points (reference
// conerf/geometry/cluster.py:73-199 Grid2DXY / Grid2DClustering, conerf/datasets/utils.py:186-206 points_in_bbox2D).
//
// The reference tests every point against one box at a time: a trimesh.transform_points pass plus an argwhere per
// box (and per x-division, and once more per expanded box), so an m x n split of a 10^7-point cloud reads the
// cloud ~3 m n times.  Here one pass transforms each point once (f64, the reference's dtype), tests it against all
// boxes, and writes the label and a box bitmask; a per-box block scan and one scatter pass turn the bitmasks into
// the ascending member lists argwhere returns.  HBM-bound integer/f64 streaming; no atomics (ballot counts per
// wave, fixed-order scans), so the lists are deterministic and in index order.
//
// k_box_test     one thread per point: frame transform, C box tests, label (last box containing the point), mask,
//                per-block per-box member counts (wave ballots, 4 waves summed in LDS)
// k_box_scan     one block per box: exclusive scan of its per-block counts, total per box
// k_box_scatter  one thread per point: member index written at box offset + block offset + wave prefix + lane rank
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blocksplit.h"

namespace gs {

namespace {

constexpr int BS_THREADS = 256;
constexpr int BS_WAVES = BS_THREADS / 64;

__device__ __forceinline__ uint64_t lanes_below() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

__global__ void __launch_bounds__(BS_THREADS) k_box_test(uint32_t N, const double* __restrict__ pts, uint32_t stride,
                                                         BoxSet bs, uint8_t* __restrict__ labels,
                                                         double* __restrict__ transformed,
                                                         uint64_t* __restrict__ masks, uint32_t* __restrict__ cnt,
                                                         uint32_t nb) {
    __shared__ uint32_t s_cnt[BS_WAVES][BOX_MAX];
    const uint32_t i = blockIdx.x * BS_THREADS + threadIdx.x;
    const bool valid = i < N;
    double x = 0.0, y = 0.0;
    if (valid) {
        const double px = pts[(size_t)i * stride], py = pts[(size_t)i * stride + 1];
        if (bs.has_T) {
            // (T0 x + T1 y) + T2 with no contraction (-ffp-contract=off): the order blocksplit_oracle.py restates
            x = (bs.T[0] * px + bs.T[1] * py) + bs.T[2];
            y = (bs.T[3] * px + bs.T[4] * py) + bs.T[5];
        } else {
            x = px;
            y = py;
        }
    }
    uint64_t mask = 0;
    uint32_t label = 0;
    const int w = threadIdx.x >> 6;
    for (uint32_t k = 0; k < bs.C; k++) {
        const double* b = bs.box[k];
        const bool in = valid && b[0] <= x && x <= b[2] && b[1] <= y && y <= b[3];
        if (in) {
            mask |= 1ull << k;
            label = k;
        }
        const uint64_t bal = __ballot(in);
        if ((threadIdx.x & 63) == 0) s_cnt[w][k] = (uint32_t)__popcll(bal);
    }
    if (valid) {
        masks[i] = mask;
        if (labels) labels[i] = (uint8_t)label;
        if (transformed) {
            transformed[2 * (size_t)i] = x;
            transformed[2 * (size_t)i + 1] = y;
        }
    }
    __syncthreads();
    if (threadIdx.x < bs.C) {
        uint32_t s = 0;
        for (int v = 0; v < BS_WAVES; v++) s += s_cnt[v][threadIdx.x];
        cnt[(size_t)threadIdx.x * nb + blockIdx.x] = s;  // box-major: each box's block counts contiguous
    }
}

__global__ void __launch_bounds__(BS_THREADS) k_box_scan(uint32_t* __restrict__ cnt, uint32_t nb,
                                                         uint32_t* __restrict__ total) {
    __shared__ uint32_t s[BS_THREADS];
    uint32_t* c = cnt + (size_t)blockIdx.x * nb;
    const uint32_t per = (nb + BS_THREADS - 1) / BS_THREADS;
    const uint32_t lo = min(threadIdx.x * per, nb), hi = min(lo + per, nb);
    uint32_t local = 0;
    for (uint32_t j = lo; j < hi; j++) local += c[j];
    s[threadIdx.x] = local;
    __syncthreads();
    for (int d = 1; d < BS_THREADS; d <<= 1) {  // inclusive Hillis-Steele scan of the per-thread sums
        const uint32_t v = threadIdx.x >= (uint32_t)d ? s[threadIdx.x - d] : 0u;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = s[threadIdx.x] - local;
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t v = c[j];
        c[j] = run;
        run += v;
    }
    if (threadIdx.x == BS_THREADS - 1) total[blockIdx.x] = s[BS_THREADS - 1];
}

__global__ void __launch_bounds__(BS_THREADS) k_box_scatter(uint32_t N, const uint64_t* __restrict__ masks,
                                                            const uint32_t* __restrict__ cnt, uint32_t nb,
                                                            BoxOffsets off, uint32_t* __restrict__ members) {
    __shared__ uint32_t s_cnt[BS_WAVES][BOX_MAX];
    const uint32_t i = blockIdx.x * BS_THREADS + threadIdx.x;
    const uint64_t mask = i < N ? masks[i] : 0ull;
    const int w = threadIdx.x >> 6;
    for (uint32_t k = 0; k < off.C; k++) {
        const uint64_t bal = __ballot((mask >> k) & 1ull);
        if ((threadIdx.x & 63) == 0) s_cnt[w][k] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    const uint64_t below = lanes_below();
    for (uint32_t k = 0; k < off.C; k++) {
        const bool in = (mask >> k) & 1ull;
        const uint64_t bal = __ballot(in);
        if (in) {
            uint32_t pos = off.first[k] + cnt[(size_t)k * nb + blockIdx.x];
            for (int v = 0; v < w; v++) pos += s_cnt[v][k];
            members[pos + (uint32_t)__popcll(bal & below)] = i;
        }
    }
}

}  // namespace

uint32_t box_blocks(uint32_t N) { return (N + BS_THREADS - 1) / BS_THREADS; }

void launch_box_test(uint32_t N, const double* pts, uint32_t stride, const BoxSet& bs, uint8_t* labels,
                     double* transformed, uint64_t* masks, uint32_t* cnt, hipStream_t s) {
    const uint32_t nb = box_blocks(N);
    if (nb) k_box_test<<<nb, BS_THREADS, 0, s>>>(N, pts, stride, bs, labels, transformed, masks, cnt, nb);
}
void launch_box_scan(uint32_t N, uint32_t C, uint32_t* cnt, uint32_t* total, hipStream_t s) {
    k_box_scan<<<C, BS_THREADS, 0, s>>>(cnt, box_blocks(N), total);
}
void launch_box_scatter(uint32_t N, const uint64_t* masks, const uint32_t* cnt, const BoxOffsets& off,
                        uint32_t* members, hipStream_t s) {
    const uint32_t nb = box_blocks(N);
    if (nb) k_box_scatter<<<nb, BS_THREADS, 0, s>>>(N, masks, cnt, nb, off, members);
}

}  // namespace gs

// Microbenchmark: device-scope atomicAdd-with-return throughput for an atomic counting sort of instances by
// tile (2.09e6 instances over 8160 tiles), as an alternative to the two-pass radix tile sort.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_atomic.hip -o tools/ubench_atomic
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime.h>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_zero(uint32_t* c, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = 0;
}
__global__ void k_count(const uint32_t* __restrict__ tile, uint32_t* __restrict__ cnt, uint32_t* __restrict__ slot, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) slot[i] = atomicAdd(&cnt[tile[i]], 1u);
}
__global__ void k_count_noret(const uint32_t* __restrict__ tile, uint32_t* __restrict__ cnt, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&cnt[tile[i]], 1u);
}

template <typename F>
float time_it(F&& f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
}

int main() {
    const int n = 2088952, T = 8160;
    std::mt19937 rng(7);
    std::vector<uint32_t> rnd(n), coh(n);
    std::uniform_int_distribution<uint32_t> ut(0, T - 1);
    for (auto& x : rnd) x = ut(rng);
    // coherent: runs of a Gaussian's rect (~6x6 tiles) as the emit writes them
    for (int i = 0; i < n;) {
        const int x0 = ut(rng) % 114, y0 = ut(rng) % 62;
        for (int y = y0; y < y0 + 6 && i < n; y++)
            for (int x = x0; x < x0 + 6 && i < n; x++) coh[i++] = y * 120 + x;
    }
    uint32_t *tile, *cnt, *slot;
    CK(hipMalloc(&tile, 4 * n)); CK(hipMalloc(&cnt, 4 * T)); CK(hipMalloc(&slot, 4 * n));
    const char* names[2] = {"random tiles", "rect-coherent"};
    std::vector<uint32_t>* srcs[2] = {&rnd, &coh};
    for (int v = 0; v < 2; v++) {
        CK(hipMemcpy(tile, srcs[v]->data(), 4 * n, hipMemcpyHostToDevice));
        const float tz = time_it([&] { k_zero<<<(T + 255) / 256, 256>>>(cnt, T); }, 20);
        const float t1 = time_it([&] {
            k_zero<<<(T + 255) / 256, 256>>>(cnt, T);
            k_count<<<(n + 255) / 256, 256>>>(tile, cnt, slot, n);
        }, 20);
        const float t2 = time_it([&] {
            k_zero<<<(T + 255) / 256, 256>>>(cnt, T);
            k_count_noret<<<(n + 255) / 256, 256>>>(tile, cnt, n);
        }, 20);
        std::vector<uint32_t> h(T);
        CK(hipMemcpy(h.data(), cnt, 4 * T, hipMemcpyDeviceToHost));
        long s = 0;
        for (auto x : h) s += x;
        printf("%-14s n=%d tiles=%d  zero %.1f us  count+slot %.1f us  count(no return) %.1f us  sum ok=%d\n", names[v], n, T,
               tz, t1 - tz, t2 - tz, (int)(s == n));
    }
    return 0;
}

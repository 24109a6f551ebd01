// Microbenchmark: per-tile instance counting with device-scope atomics (one counter array) vs XCD-local counters
// (one counter array per XCD, indexed by the wave's XCC id, workgroup-scope atomics resolved in that XCD's L2).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_xcc_atomic.hip -o gpurun_out/ubench_xcc_atomic
#include <stdio.h>
#include <stdlib.h>
#include <hip/hip_runtime.h>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7u;
}
__global__ void k_zero(uint32_t* c, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = 0;
}
__global__ void k_dev(const uint32_t* __restrict__ tile, uint32_t* __restrict__ cnt, uint32_t* __restrict__ slot, int n, int ret) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (ret) slot[i] = atomicAdd(&cnt[tile[i]], 1u);
    else atomicAdd(&cnt[tile[i]], 1u);
}
__global__ void k_xcc(const uint32_t* __restrict__ tile, uint32_t* __restrict__ cnt8, uint32_t* __restrict__ slot, int n, int T,
                      int ret, uint32_t* __restrict__ who) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = xcc_id();
    uint32_t* c = cnt8 + (size_t)x * T + tile[i];
    if (ret) {
        slot[i] = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        who[i] = x;
    } else {
        __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
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
    const int n = 1835850, T = 8160;
    std::mt19937 rng(7);
    std::vector<uint32_t> rnd(n), coh(n);
    std::uniform_int_distribution<uint32_t> ut(0, T - 1);
    for (auto& x : rnd) x = ut(rng);
    for (int i = 0; i < n;) {  // runs of a Gaussian's rect (~6x6 tiles) as the emission writes them
        const int x0 = ut(rng) % 114, y0 = ut(rng) % 62;
        for (int y = y0; y < y0 + 6 && i < n; y++)
            for (int x = x0; x < x0 + 6 && i < n; x++) coh[i++] = y * 120 + x;
    }
    uint32_t *tile, *cnt, *slot, *who;
    CK(hipMalloc(&tile, 4 * n)); CK(hipMalloc(&cnt, 4 * 8 * T)); CK(hipMalloc(&slot, 4 * n)); CK(hipMalloc(&who, 4 * n));
    const char* names[2] = {"random tiles", "rect-coherent"};
    std::vector<uint32_t>* srcs[2] = {&rnd, &coh};
    for (int v = 0; v < 2; v++) {
        CK(hipMemcpy(tile, srcs[v]->data(), 4 * n, hipMemcpyHostToDevice));
        const int nb = (n + 255) / 256;
        const float tz = time_it([&] { k_zero<<<(8 * T + 255) / 256, 256>>>(cnt, 8 * T); }, 20);
        float t[4];
        for (int ret = 0; ret < 2; ret++) {
            t[ret] = time_it([&] { k_zero<<<(8 * T + 255) / 256, 256>>>(cnt, 8 * T); k_dev<<<nb, 256>>>(tile, cnt, slot, n, ret); }, 20) - tz;
            t[2 + ret] = time_it([&] { k_zero<<<(8 * T + 255) / 256, 256>>>(cnt, 8 * T); k_xcc<<<nb, 256>>>(tile, cnt, slot, n, T, ret, who); }, 20) - tz;
        }
        // check: per tile, the 8 XCD counts sum to the instance count, and every (xcc, tile) slot set is 0..c-1
        std::vector<uint32_t> h(8 * T), s(n), w(n);
        CK(hipMemcpy(h.data(), cnt, 4 * 8 * T, hipMemcpyDeviceToHost));
        CK(hipMemcpy(s.data(), slot, 4 * n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(w.data(), who, 4 * n, hipMemcpyDeviceToHost));
        std::vector<uint32_t> per(T, 0), used_x(8, 0);
        long bad = 0;
        for (int i = 0; i < n; i++) { per[(*srcs[v])[i]]++; used_x[w[i]]++; if (s[i] >= h[(size_t)w[i] * T + (*srcs[v])[i]]) bad++; }
        for (int tt = 0; tt < T; tt++) { uint32_t q = 0; for (int x = 0; x < 8; x++) q += h[(size_t)x * T + tt]; if (q != per[tt]) bad++; }
        printf("%-14s n=%d tiles=%d  device: %.1f us (no return) %.1f us (return)   xcd-local: %.1f us (no return) %.1f us (return)  bad=%ld  per-xcc",
               names[v], n, T, t[0], t[1], t[2], t[3], bad);
        for (int x = 0; x < 8; x++) printf(" %u", used_x[x]);
        printf("\n");
    }
    return 0;
}

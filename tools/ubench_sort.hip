// Microbenchmark: the in-tree LSD radix sort (sortscan.hip) against rocPRIM's device radix sort on the two
// sorts of the forward (1e6 depth keys over 32 bits; 2.09e6 tile keys over 13 bits), plus the u32 scan.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_sort.hip dogs_amd/csrc/sortscan.hip -o tools/ubench_sort
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <vector>
#include <random>
#include "../dogs_amd/csrc/sortscan.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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
    return ms * 1000.f / reps;  // us
}

void run(const char* name, const std::vector<uint32_t>& hk, int end_bit) {
    const uint32_t n = (uint32_t)hk.size();
    uint32_t *k0, *v0, *k1, *v1, *kr, *vr, *kin;
    CK(hipMalloc(&k0, 4 * n)); CK(hipMalloc(&v0, 4 * n)); CK(hipMalloc(&k1, 4 * n)); CK(hipMalloc(&v1, 4 * n));
    CK(hipMalloc(&kr, 4 * n)); CK(hipMalloc(&vr, 4 * n)); CK(hipMalloc(&kin, 4 * n));
    CK(hipMemcpy(kin, hk.data(), 4 * n, hipMemcpyHostToDevice));
    std::vector<uint32_t> hidx(n);
    for (uint32_t i = 0; i < n; i++) hidx[i] = i;
    uint32_t* vin;
    CK(hipMalloc(&vin, 4 * n));
    CK(hipMemcpy(vin, hidx.data(), 4 * n, hipMemcpyHostToDevice));
    void* tmp;
    CK(hipMalloc(&tmp, gs::radix_sort_temp_bytes(n)));
    int which = 0;
    const float t_ours = time_it([&] {
        (void)hipMemcpyAsync(k0, kin, 4 * n, hipMemcpyDeviceToDevice, 0);
        which = gs::radix_sort_pairs(k0, v0, k1, v1, nullptr, n, 0, end_bit, tmp, 0);
    }, 20);
    const float t_copy = time_it([&] { (void)hipMemcpyAsync(k0, kin, 4 * n, hipMemcpyDeviceToDevice, 0); }, 20);
    size_t rb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, rb, kin, kr, vin, vr, n, 0, end_bit, 0));
    void* rtmp;
    CK(hipMalloc(&rtmp, rb));
    const float t_roc = time_it([&] { (void)rocprim::radix_sort_pairs(rtmp, rb, kin, kr, vin, vr, n, 0, end_bit, 0); }, 20);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> a(n), b(n), c(n), d(n);
    CK(hipMemcpy(a.data(), which ? k1 : k0, 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), which ? v1 : v0, 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), kr, 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d.data(), vr, 4 * n, hipMemcpyDeviceToHost));
    const bool same = a == c && b == d;
    printf("%-22s n=%8u bits=%2d  ours %7.1f us (incl. %5.1f us key copy)  rocprim %7.1f us  same=%d\n", name, n, end_bit,
           t_ours, t_copy, t_roc, (int)same);
    // scan (u32), no gather
    uint32_t* tot;
    CK(hipMalloc(&tot, 4));
    void* stmp;
    CK(hipMalloc(&stmp, gs::scan_temp_bytes(n)));
    std::vector<uint32_t> small(n);
    for (uint32_t i = 0; i < n; i++) small[i] = hk[i] & 31u;
    CK(hipMemcpy(k0, small.data(), 4 * n, hipMemcpyHostToDevice));
    const float s_ours = time_it([&] { gs::exclusive_scan(k0, n, k1, tot, stmp, 0); }, 20);
    size_t sb = 0;
    CK(rocprim::exclusive_scan(nullptr, sb, k0, kr, 0u, n, rocprim::plus<uint32_t>(), 0));
    void* s2;
    CK(hipMalloc(&s2, sb));
    const float s_roc = time_it([&] { (void)rocprim::exclusive_scan(s2, sb, k0, kr, 0u, n, rocprim::plus<uint32_t>(), 0); }, 20);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a.data(), k1, 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), kr, 4 * n, hipMemcpyDeviceToHost));
    printf("%-22s scan ours %7.1f us  rocprim %7.1f us  same=%d\n", name, s_ours, s_roc, (int)(a == c));
    CK(hipFree(k0)); CK(hipFree(v0)); CK(hipFree(k1)); CK(hipFree(v1)); CK(hipFree(kr)); CK(hipFree(vr));
    CK(hipFree(kin)); CK(hipFree(vin)); CK(hipFree(tmp)); CK(hipFree(rtmp)); CK(hipFree(tot)); CK(hipFree(stmp));
    CK(hipFree(s2));
}

int main() {
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> uz(2.f, 20.f), u01(0.f, 1.f);
    {
        std::vector<uint32_t> k(1000000);
        for (auto& x : k) {
            const float z = uz(rng);
            uint32_t b;
            memcpy(&b, &z, 4);
            x = u01(rng) < 0.12f ? 0xffffffffu : b;
        }
        run("depth 1e6", k, 32);
    }
    {
        std::vector<uint32_t> k(5000000);
        for (auto& x : k) {
            const float z = uz(rng);
            uint32_t b;
            memcpy(&b, &z, 4);
            x = u01(rng) < 0.12f ? 0xffffffffu : b;
        }
        run("depth 5e6", k, 32);
    }
    {
        std::vector<uint32_t> k(2088952);
        std::uniform_int_distribution<uint32_t> ut(0, 8159);
        for (auto& x : k) x = ut(rng);
        run("tile 2.09e6", k, 13);
    }
    return 0;
}

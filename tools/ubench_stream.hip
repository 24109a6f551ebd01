// Streaming HBM rates on one MI355X: what an Adam-shaped kernel (3 float streams read and written in place, one more
// read) can reach, against pure reads and pure writes.  hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip -o
// /tmp/ubench_stream && /tmp/ubench_stream [floats per stream, default 59e6]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_rmw3(f4* a, f4* b, f4* c, const f4* g, size_t n4, int nt) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    f4 x, y, z, w;
    if (nt) {
        x = __builtin_nontemporal_load(a + i); y = __builtin_nontemporal_load(b + i);
        z = __builtin_nontemporal_load(c + i); w = __builtin_nontemporal_load(g + i);
    } else {
        x = a[i]; y = b[i]; z = c[i]; w = g[i];
    }
    y = y * 0.9f + w * 0.1f;
    z = z * 0.999f + w * w * 0.001f;
    x = x - 0.001f * y / (z + 1e-8f);
    if (nt) {
        __builtin_nontemporal_store(x, a + i); __builtin_nontemporal_store(y, b + i); __builtin_nontemporal_store(z, c + i);
    } else {
        a[i] = x; b[i] = y; c[i] = z;
    }
}
__global__ void __launch_bounds__(256) k_read(const f4* a, size_t n4, float* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const f4 x = __builtin_nontemporal_load(a + i);
    if (x.x == 12345.678f) out[0] = x.y;  // never true: keeps the load
}
__global__ void __launch_bounds__(256) k_write(f4* a, size_t n4) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    __builtin_nontemporal_store((f4){1.f, 2.f, 3.f, 4.f}, a + i);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? (size_t)atof(argv[1]) : (size_t)59e6;
    const size_t n4 = n / 4;
    f4 *a, *b, *c, *g;
    float* out;
    CK(hipMalloc(&a, n4 * 16)); CK(hipMalloc(&b, n4 * 16)); CK(hipMalloc(&c, n4 * 16)); CK(hipMalloc(&g, n4 * 16));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(a, 0, n4 * 16)); CK(hipMemset(b, 0, n4 * 16)); CK(hipMemset(c, 0, n4 * 16)); CK(hipMemset(g, 0, n4 * 16));
    const unsigned blocks = (unsigned)((n4 + 255) / 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 4; mode++) {
        for (int it = 0; it < 23; it++) {
            if (it == 3) CK(hipEventRecord(e0));
            if (mode == 0) k_rmw3<<<blocks, 256>>>(a, b, c, g, n4, 1);
            else if (mode == 1) k_rmw3<<<blocks, 256>>>(a, b, c, g, n4, 0);
            else if (mode == 2) k_read<<<blocks, 256>>>(a, n4, out);
            else k_write<<<blocks, 256>>>(a, n4);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 20;
        const double bytes = (mode < 2 ? 7.0 : 1.0) * n4 * 16;
        const char* name[4] = {"rmw3+1 nt", "rmw3+1 cached", "read nt", "write nt"};
        printf("%-14s %8.1f us  %7.0f GB/s  (%.0f MB per launch)\n", name[mode], us, bytes / us / 1e3, bytes / 1e6);
    }
    return 0;
}

// VALU issue-rate microbenchmark (gfx950): cycles per wave64 instruction for independent streams of
// v_fma_f32, v_pk_fma_f32 and v_exp_f32 at 8 waves/SIMD on every CU.  Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
#define ITERS 4096
__global__ void __launch_bounds__(256) k_fma(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = __builtin_fmaf(a[i], s, 0.5f);
    float r = 0; for (int i = 0; i < 8; i++) r += a[i];
    if (r == 1.2345f) out[0] = r;
}
__global__ void __launch_bounds__(256) k_pk(float* out, float s) {
    v2f a[8];
    for (int i = 0; i < 8; i++) a[i] = (v2f){threadIdx.x * 0.001f + i, i * 0.5f};
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = __builtin_elementwise_fma(a[i], (v2f){s, s}, (v2f){0.5f, 0.25f});
    float r = 0; for (int i = 0; i < 8; i++) r += a[i].x + a[i].y;
    if (r == 1.2345f) out[0] = r;
}
__global__ void __launch_bounds__(256) k_exp(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * -0.001f - i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = __builtin_amdgcn_exp2f(a[i]) * s;  // exp + mul
    float r = 0; for (int i = 0; i < 8; i++) r += a[i];
    if (r == 1.2345f) out[0] = r;
}
__global__ void __launch_bounds__(256) k_mul(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * -0.001f - i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = (a[i] * s) * s;  // 2 muls
    float r = 0; for (int i = 0; i < 8; i++) r += a[i];
    if (r == 1.2345f) out[0] = r;
}
template <typename K>
static void run(const char* name, K k, int instr_per_iter) {
    float* out; (void)hipMalloc(&out, 4);
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU -> 8 waves/SIMD
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<<<blocks, 256>>>(out, 1.0001f);
    (void)hipEventRecord(e0);
    k<<<blocks, 256>>>(out, 1.0001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0;
    const double instr = waves * ITERS * 8.0 * instr_per_iter;  // wave-instructions
    const double simds = 1024.0;
    int clk = 0; (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
    const double cyc = ms * 1e-3 * clk * 1e3 * simds / instr;
    printf("%-8s %.3f ms  %.2f cycles per wave-instruction per SIMD (clock %d MHz)\n", name, ms, cyc, clk / 1000);
    (void)hipFree(out);
}
int main() {
    run("fma", k_fma, 1);
    run("pk_fma", k_pk, 1);
    run("mul", k_mul, 2);
    run("exp+mul", k_exp, 2);
    return 0;
}

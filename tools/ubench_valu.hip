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
// one dependent chain per wave (no ILP)
__global__ void __launch_bounds__(256) k_fma_dep(float* out, float s) {
    float a = threadIdx.x * 0.001f;
    for (int it = 0; it < ITERS * 8; it++) a = __builtin_fmaf(a, s, 0.5f);
    if (a == 1.2345f) out[0] = a;
}
__global__ void __launch_bounds__(256) k_pk_dep(float* out, float s) {
    v2f a = (v2f){threadIdx.x * 0.001f, 0.5f};
    for (int it = 0; it < ITERS * 8; it++) a = __builtin_elementwise_fma(a, (v2f){s, s}, (v2f){0.5f, 0.25f});
    if (a.x + a.y == 1.2345f) out[0] = a.x;
}
__global__ void __launch_bounds__(256) k_exp_dep(float* out, float s) {
    float a = threadIdx.x * -0.001f;
    for (int it = 0; it < ITERS * 8; it++) a = __builtin_amdgcn_exp2f(a) * s - 1.5f;  // exp, fma
    if (a == 1.2345f) out[0] = a;
}
// 2 chains per wave
__global__ void __launch_bounds__(256) k_fma_dep2(float* out, float s) {
    float a = threadIdx.x * 0.001f, b = a + 1.0f;
    for (int it = 0; it < ITERS * 4; it++) { a = __builtin_fmaf(a, s, 0.5f); b = __builtin_fmaf(b, s, 0.25f); }
    if (a + b == 1.2345f) out[0] = a;
}
// compare -> select (v_cmp_*_e64 to an SGPR pair + v_cndmask_b32_e64), 8 independent lanes of work
__global__ void __launch_bounds__(256) k_cmpsel(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) {
            float v;
            asm volatile("v_cmp_lt_f32_e64 s[20:21], %1, %2\n\tv_cndmask_b32_e64 %0, %1, 0, s[20:21]"
                         : "=v"(v) : "v"(a[i]), "s"(s) : "s20", "s21");
            a[i] = v + 0.0f;
        }
    float r = 0; for (int i = 0; i < 8; i++) r += a[i];
    if (r == 1.2345f) out[0] = r;
}
// min (v_min_f32 with literal), 8 independent chains
__global__ void __launch_bounds__(256) k_min(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) {
            asm volatile("v_min_f32_e32 %0, 0x3f7d70a4, %0\n\tv_max_f32_e32 %0, s%1, %0" : "+v"(a[i]) : "n"(0) );
        }
    float r = 0; for (int i = 0; i < 8; i++) r += a[i];
    if (r == 1.2345f) out[0] = r;
}
// v_cndmask_b32_e32 (vcc) alone
__global__ void __launch_bounds__(256) k_cnd(float* out, float s) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 0.001f + i;
    asm volatile("v_cmp_lt_f32_e32 vcc, 0.5, %0" :: "v"(a[0]) : "vcc");
    for (int it = 0; it < ITERS; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_cndmask_b32_e32 %0, 0, %0, vcc" : "+v"(a[i]));
    float r = 0; for (int i = 0; i < 8; i++) r += a[i];
    if (r == 1.2345f) out[0] = r;
}
// v_cmp_*_e64 to SGPR pairs alone (8 distinct destinations)
__global__ void __launch_bounds__(256) k_cmp(float* out, float s) {
    float a = threadIdx.x * 0.001f;
    for (int it = 0; it < ITERS; it++)
        asm volatile("v_cmp_lt_f32_e64 s[20:21], %0, 1.0\n\tv_cmp_lt_f32_e64 s[22:23], %0, 2.0\n\t"
                     "v_cmp_lt_f32_e64 s[24:25], %0, 0.5\n\tv_cmp_lt_f32_e64 s[26:27], %0, 4.0\n\t"
                     "v_cmp_lt_f32_e64 s[28:29], %0, 1.0\n\tv_cmp_lt_f32_e64 s[30:31], %0, 2.0\n\t"
                     "v_cmp_lt_f32_e64 s[32:33], %0, 0.5\n\tv_cmp_lt_f32_e64 s[34:35], %0, 4.0"
                     :: "v"(a) : "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35");
    if (a == 1.2345f) out[0] = a;
}
// SALU: s_and_b64 chain on 8 independent pairs
__global__ void __launch_bounds__(256) k_salu(float* out, float s) {
    for (int it = 0; it < ITERS; it++)
        asm volatile("s_and_b64 s[20:21], s[20:21], s[22:23]\n\ts_or_b64 s[24:25], s[24:25], s[26:27]\n\t"
                     "s_and_b64 s[28:29], s[28:29], s[30:31]\n\ts_or_b64 s[32:33], s[32:33], s[34:35]\n\t"
                     "s_andn2_b64 s[36:37], s[36:37], s[38:39]\n\ts_or_b64 s[40:41], s[40:41], s[42:43]\n\t"
                     "s_and_b64 s[44:45], s[44:45], s[46:47]\n\ts_or_b64 s[48:49], s[48:49], s[50:51]"
                     ::: "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30","s31","s32","s33","s34","s35",
                         "s36","s37","s38","s39","s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51");
    if (s == 1.2345f) out[0] = s;
}
template <typename K>
static void run(const char* name, K k, int instr_per_iter, int waves_per_simd = 8) {
    float* out; (void)hipMalloc(&out, 4);
    const int blocks = 256 * waves_per_simd;  // blocks of 4 waves, one per SIMD
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
    run("cmp+sel", k_cmpsel, 3);   // cmp, cndmask, add
    run("min+max", k_min, 2);
    run("cnd_vcc", k_cnd, 1);
    run("cmp_e64", k_cmp, 1);
    run("salu_b64", k_salu, 1);
    for (int w : {8, 4, 2}) {
        printf("-- dependent chains, %d waves/SIMD\n", w);
        run("fma_dep", k_fma_dep, 1, w);
        run("fma_dep2", k_fma_dep2, 1, w);
        run("pk_dep", k_pk_dep, 1, w);
        run("exp_fma", k_exp_dep, 2, w);
    }
    return 0;
}

// Throughput of the VALU instructions the scorer uses (one value per kernel:
// ns per wave-instruction per CU, all CUs busy).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N_IT 4096
template <int OP>
__global__ __launch_bounds__(256) void kb(uint32_t* out, uint32_t seed, int sl) {
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
    const uint32_t x = seed * 0x9E3779B9u + threadIdx.x;
    for (int it = 0; it < N_IT; ++it) {
#define STEP(a) \
        if (OP == 0) a = __builtin_amdgcn_udot4(x, a, a, false); \
        if (OP == 1) a = __builtin_amdgcn_sad_u8(x, a, a); \
        if (OP == 2) a = __builtin_amdgcn_alignbyte(x, a, sl); \
        if (OP == 3) a = a + x; \
        if (OP == 4) a = __builtin_amdgcn_readlane(a, sl) + a; \
        if (OP == 5) a = __builtin_amdgcn_udot4(x, (uint32_t)sl, a, false); \
        if (OP == 6) a = (uint32_t)__builtin_amdgcn_sdot4((int)x, (int)a, (int)a, false); \
        if (OP == 7) a = __builtin_amdgcn_ubfe(a, sl, 8) + a; \
        if (OP == 8) a = (uint32_t)__mul24((int)a, (int)x); \
        if (OP == 9) a = __builtin_bit_cast(uint32_t, __builtin_amdgcn_rsqf(__builtin_bit_cast(float, a))); \
        if (OP == 10) a = __builtin_bit_cast(uint32_t, fmaf(__builtin_bit_cast(float, a), 1.0001f, 0.5f)); \
        if (OP == 11) { typedef unsigned short v2u16 __attribute__((ext_vector_type(2))); \
                        a = __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u16, a) + __builtin_bit_cast(v2u16, x)); }
        STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
template <int OP>
__global__ __launch_bounds__(256) void kd(double* out, double seed) {
    double a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int it = 0; it < N_IT; ++it) {
#define STEPD(a) if (OP == 0) a = fma(a, seed, 0.5); if (OP == 1) a = a / seed; if (OP == 2) a = sqrt(a); \
        if (OP == 3) a = a * seed; if (OP == 4) a = (double)(int)__builtin_bit_cast(uint64_t, a) + a; \
        if (OP == 5) a = __builtin_amdgcn_rsq(a);
        STEPD(a0) STEPD(a1) STEPD(a2) STEPD(a3) STEPD(a4) STEPD(a5) STEPD(a6) STEPD(a7)
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
template <class K, class... A>
void run(const char* name, K k, int ninstr, A... args) {
    const int blocks = 256 * 8;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, args...);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, args...);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0 * 5;
    const double instr = waves * N_IT * 8 * ninstr;
    // cycles per wave-instruction per SIMD, assuming 2.4 GHz and 1024 SIMDs
    const double cyc = ms * 1e-3 * 2.4e9 * 1024 / instr;
    printf("%-12s %8.3f ms  %.2f SIMD-cycles per wave-instruction\n", name, ms, cyc);
}
int main() {
    uint32_t* o; double* od;
    hipMalloc(&o, 256 * 8 * 256 * 4); hipMalloc(&od, 256 * 8 * 256 * 8);
    run("dot4_u8", kb<0>, 1, o, 7u, 1);
    run("sad_u8", kb<1>, 1, o, 7u, 1);
    run("alignbyte", kb<2>, 1, o, 7u, 1);
    run("add_u32", kb<3>, 1, o, 7u, 1);
    run("readlane+add", kb<4>, 2, o, 7u, 1);
    run("dot4 sgpr", kb<5>, 1, o, 7u, 1);
    run("sdot4_i8", kb<6>, 1, o, 7u, 1);
    run("bfe+add", kb<7>, 2, o, 7u, 1);
    run("mul_i24", kb<8>, 1, o, 7u, 1);
    run("rsq_f32", kb<9>, 1, o, 7u, 1);
    run("fma_f32", kb<10>, 1, o, 7u, 1);
    run("pk_add_u16", kb<11>, 1, o, 7u, 1);
    run("fma_f64", kd<0>, 1, od, 1.0000001);
    run("mul_f64", kd<3>, 1, od, 1.0000001);
    run("cvt_f64_i32+add", kd<4>, 2, od, 1.0000001);
    run("rsq_f64", kd<5>, 1, od, 1.0000001);
    run("div_f64", kd<1>, 1, od, 1.0000001);
    run("sqrt_f64", kd<2>, 1, od, 1.0000001);
    return 0;
}

// Checks the operand/result lane maps the MFMA scorers rely on, with exact
// integer data, for v_mfma_i32_16x16x64_i8 and v_mfma_i32_16x16x32_i8 on gfx950:
//   A: lane l holds A[m = l&15][k = KB(l>>4) + j], j = byte 0..KB-1 of its operand
//   B: lane l holds B[k = KB(l>>4) + j][n = l&15]
//   D: lane l holds D[m = 4(l>>4) + i][n = l&15], i = 0..3
// (KB = 16 for x64, 8 for x32), and times back-to-back issue of each (one wave
// per SIMD, four independent accumulators).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int K>
__global__ void k_mfma(const int8_t* A, const int8_t* B, int32_t* D) {
    constexpr int KB = K / 4;
    const int l = threadIdx.x, m = l & 15, h = l >> 4;
    int8_t a[16] = {}, b[16] = {};
    for (int j = 0; j < KB; ++j) {
        a[j] = A[m * K + KB * h + j];
        b[j] = B[(KB * h + j) * 16 + m];
    }
    v4i acc = {0, 0, 0, 0};
    if constexpr (K == 64) {
        v4i av, bv;
        __builtin_memcpy(&av, a, 16);
        __builtin_memcpy(&bv, b, 16);
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
    } else {
        long av, bv;
        __builtin_memcpy(&av, a, 8);
        __builtin_memcpy(&bv, b, 8);
        acc = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, acc, 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i) D[(4 * h + i) * 16 + m] = acc[i];
}

template <int K>
__global__ void k_rate(int iters, int32_t* out, unsigned long long* cyc) {
    v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const int l = threadIdx.x;
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        if constexpr (K == 64) {
            const v4i a = {l + it, l, it, 1}, b = {l, it, 3, l};
            c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
        } else {
            const long a = (long)(l + it) << 8 | 7, b = (long)l * 3 + it;
            c0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c3, 0, 0, 0);
        }
    }
    const unsigned long long t1 = clock64();
    const v4i s = c0 + c1 + c2 + c3;
    out[blockIdx.x * 64 + l] = s[0] + s[1] + s[2] + s[3];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
int check(const char* name) {
    int8_t hA[16 * 64], hB[64 * 16];
    for (int i = 0; i < 16 * K; ++i) {
        hA[i] = (int8_t)(rand() & 0xff);
        hB[i] = (int8_t)(rand() & 0xff);
    }
    int8_t *dA, *dB;
    int32_t* dD;
    int32_t hD[256];
    (void)hipMalloc(&dA, 1024);
    (void)hipMalloc(&dB, 1024);
    (void)hipMalloc(&dD, 1024);
    (void)hipMemcpy(dA, hA, 16 * K, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 16 * K, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma<K>, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    if (hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            int32_t ref = 0;
            for (int k = 0; k < K; ++k) ref += (int32_t)hA[m * K + k] * (int32_t)hB[k * 16 + n];
            if (ref != hD[m * 16 + n]) {
                std::printf("%s MISMATCH m=%d n=%d got %d want %d\n", name, m, n, hD[m * 16 + n], ref);
                return 1;
            }
        }
    // issue rate: 1024 workgroups of one wave (several per SIMD), 4 MFMAs per iteration
    int32_t* dout;
    unsigned long long* dcyc;
    const int blocks = 1024, iters = 4096;
    (void)hipMalloc(&dout, blocks * 64 * 4);
    (void)hipMalloc(&dcyc, blocks * 8);
    hipLaunchKernelGGL(k_rate<K>, dim3(1), dim3(64), 0, 0, iters, dout, dcyc);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
    std::printf("%s layout ok; one wave alone: %.1f cycles per MFMA\n", name, (double)c / (4.0 * iters));
    return 0;
}

int main() {
    srand(7);
    int rc = check<64>("mfma_i32_16x16x64_i8");
    if (rc) return rc;
    rc = check<32>("mfma_i32_16x16x32_i8");
    if (rc) return rc;
    std::printf("mfma_layout ok\n");
    return 0;
}

// Checks the operand/result lane maps k_score_mfma relies on for
// v_mfma_i32_16x16x64_i8 on gfx950, with exact integer data:
//   A: lane l holds A[m = l&15][k = 16(l>>4) + j], j = byte 0..15 of its 4 dwords
//   B: lane l holds B[k = 16(l>>4) + j][n = l&15]
//   D: lane l holds D[m = 4(l>>4) + i][n = l&15], i = 0..3
// Prints "mfma_layout ok" or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_mfma(const int8_t* A, const int8_t* B, int32_t* D) {
    const int l = threadIdx.x, m = l & 15, h = l >> 4;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[m * 64 + 16 * h + j];     // A row-major [16][64]
        b[j] = B[(16 * h + j) * 16 + m];   // B row-major [64][16], n = l & 15
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[(4 * h + i) * 16 + m] = acc[i];
}

int main() {
    int8_t hA[16 * 64], hB[64 * 16];
    srand(7);
    for (int i = 0; i < 1024; ++i) {
        hA[i] = (int8_t)(rand() & 0xff);
        hB[i] = (int8_t)(rand() & 0xff);
    }
    int8_t *dA, *dB;
    int32_t* dD;
    int32_t hD[256];
    (void)hipMalloc(&dA, 1024);
    (void)hipMalloc(&dB, 1024);
    (void)hipMalloc(&dD, 1024);
    (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    if (hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            int32_t ref = 0;
            for (int k = 0; k < 64; ++k) ref += (int32_t)hA[m * 64 + k] * (int32_t)hB[k * 16 + n];
            if (ref != hD[m * 16 + n]) {
                std::printf("mfma_layout MISMATCH m=%d n=%d got %d want %d\n", m, n, hD[m * 16 + n], ref);
                return 1;
            }
        }
    std::printf("mfma_layout ok\n");
    return 0;
}

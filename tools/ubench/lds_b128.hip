// Does ds_read_b128 at a 4-byte (not 16-byte) aligned LDS address return the
// right dwords on gfx950, and what does it cost against dword reads?
// Diagnostic only (decides whether a row-contiguous LDS layout can serve a
// window row with one 16-byte read).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int LDS_DW = 16384;   // 64 KB

__global__ __launch_bounds__(256) void k_check(uint32_t* bad, int off, int stride) {
    __shared__ uint32_t lds[LDS_DW];
    for (int i = threadIdx.x; i < LDS_DW; i += 256) lds[i] = i * 2654435761u;
    __syncthreads();
    const int dw = ((threadIdx.x * stride) % (LDS_DW - 64)) + off;
    const uint32_t addr = dw * 4;
    u4 v;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    int b = 0;
    for (int k = 0; k < 4; ++k)
        if (v[k] != (uint32_t)(dw + k) * 2654435761u) b = 1;
    if (b) atomicAdd(bad, 1);
}

// MODE 0: four ds_read_b128 at dword offset `off` (+0, +64, +128, +192 dwords)
// MODE 1: the same 64 bytes per lane as eight ds_read2_b32
template <int MODE>
__global__ __launch_bounds__(256) void k_time(uint32_t* out, int off, int stride, int iters) {
    __shared__ uint32_t lds[LDS_DW];
    for (int i = threadIdx.x; i < LDS_DW; i += 256) lds[i] = i;
    __syncthreads();
    uint32_t acc = 0;
    const int lane_dw = ((threadIdx.x & 63) * stride) % (LDS_DW - 8192);
    for (int it = 0; it < iters; ++it) {
        const int dw = lane_dw + ((it * 37) & 4095) + off;
        const uint32_t addr = dw * 4;
        if (MODE == 0) {
            u4 v0, v1, v2, v3;
            asm volatile("ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:256\n"
                         " ds_read_b128 %2, %4 offset:512\n ds_read_b128 %3, %4 offset:768\n s_waitcnt lgkmcnt(0)"
                         : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3) : "v"(addr) : "memory");
            acc += v0[0] ^ v1[1] ^ v2[2] ^ v3[3];
        } else {
            unsigned long long p0, p1, p2, p3, p4, p5, p6, p7;
            asm volatile("ds_read2_b32 %0, %8 offset1:1\n ds_read2_b32 %1, %8 offset0:2 offset1:3\n"
                         " ds_read2_b32 %2, %8 offset0:64 offset1:65\n ds_read2_b32 %3, %8 offset0:66 offset1:67\n"
                         " ds_read2_b32 %4, %8 offset0:128 offset1:129\n ds_read2_b32 %5, %8 offset0:130 offset1:131\n"
                         " ds_read2_b32 %6, %8 offset0:192 offset1:193\n ds_read2_b32 %7, %8 offset0:194 offset1:195\n"
                         " s_waitcnt lgkmcnt(0)"
                         : "=v"(p0), "=v"(p1), "=v"(p2), "=v"(p3), "=v"(p4), "=v"(p5), "=v"(p6), "=v"(p7)
                         : "v"(addr) : "memory");
            acc += (uint32_t)(p0 ^ p1 ^ p2 ^ p3 ^ p4 ^ p5 ^ p6 ^ p7);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    uint32_t *bad, *out;
    hipMalloc(&bad, 4);
    hipMalloc(&out, 4 * 256 * 4096);
    for (int off = 0; off < 4; ++off)
        for (int stride : {4, 37, 148}) {
            hipMemset(bad, 0, 4);
            hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, 0, bad, off, stride);
            uint32_t h = 0;
            hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
            printf("check off %d stride %3d: %u of 256 lanes wrong\n", off, stride, h);
        }
    const int iters = 4096, blocks = 256 * 8;
    for (int mode = 0; mode < 2; ++mode)
        for (int off = 0; off < 2; ++off)
            for (int stride : {4, 148}) {
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                auto k = mode == 0 ? k_time<0> : k_time<1>;
                hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, off, stride, iters);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, off, stride, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                // CU-cycles per wave-read of 16 B/lane (256 CUs, 2.4 GHz)
                const double waves = blocks * 4.0;
                printf("mode %s off %d stride %3d: %.3f ms, %.2f CU-cycles per 16-B/lane wave read\n",
                       mode == 0 ? "b128 " : "2xrd2", off, stride, ms, ms * 1e-3 * 2.4e9 * 256 / (waves * iters * 4));
            }
    return 0;
}

// LDS read cost on gfx950 for the scorer's access shapes (diagnostic only):
//   rd2   : ds_read2_b32, lane stride 1 dword, two dwords 64 dwords apart
//           (k_score_tiled3's own-window reads today: 8 B per lane)
//   b64   : ds_read_b64, lane stride 2 dwords (8-B aligned, 8 B per lane)
//   b64u  : ds_read_b64 at a 4-B (not 8-B) aligned address, lane stride 2
//   rd2bc : ds_read2_b32, every lane the same address (reference broadcast)
//   b64bc : ds_read_b64, every lane the same address
//   b32s2 : ds_read_b32, lane stride 2 dwords (2-way bank conflict expected)
// Each prints whether the returned dwords are right and the CU-cycles per
// wave-instruction with 16 reads in flight, 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int LDS_DW = 4096;   // 16 KB: 4 workgroups of 4 waves per CU

using lds_ptr = __attribute__((address_space(3))) uint32_t*;

__device__ inline uint32_t lds_addr(uint32_t* p) {
    return (uint32_t)(uintptr_t)(lds_ptr)p;
}

template <int MODE>
__device__ inline void rd(uint32_t a, uint32_t& x, uint32_t& y) {
    unsigned long long v;
    if (MODE == 0 || MODE == 3) {
        asm volatile("ds_read2_b32 %0, %1 offset1:64" : "=v"(v) : "v"(a));
    } else if (MODE == 5) {
        uint32_t w;
        asm volatile("ds_read_b32 %0, %1" : "=v"(w) : "v"(a));
        v = w;
    } else {
        asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
    }
    x = (uint32_t)v;
    y = (uint32_t)(v >> 32);
}

template <int MODE>
__device__ inline uint32_t lane_dw(int lane) {
    if (MODE == 0) return lane;
    if (MODE == 1) return 2 * lane;
    if (MODE == 2) return 2 * lane + 1;
    if (MODE == 5) return 2 * lane;
    return 38;   // broadcast (8-B aligned)
}

template <int MODE>
__global__ __launch_bounds__(256) void k_check(uint32_t* bad) {
    __shared__ uint32_t lds[LDS_DW];
    for (int i = threadIdx.x; i < LDS_DW; i += 256) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t dw = lane_dw<MODE>(threadIdx.x & 63) + 256 * (threadIdx.x >> 6);
    uint32_t x, y;
    rd<MODE>(lds_addr(lds) + dw * 4, x, y);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t dy = (MODE == 0 || MODE == 3) ? dw + 64 : dw + 1;
    int b = x != dw * 2654435761u;
    if (MODE != 5 && y != dy * 2654435761u) b = 1;
    if (b) atomicAdd(bad, 1);
    if (threadIdx.x == 0) lds[0] = 0;   // keep the fill alive
}

template <int MODE>
__global__ __launch_bounds__(256) void k_time(uint32_t* out, int iters) {
    __shared__ uint32_t lds[LDS_DW];
    for (int i = threadIdx.x; i < LDS_DW; i += 256) lds[i] = i;
    __syncthreads();
    const uint32_t base = lds_addr(lds) + 4 * (lane_dw<MODE>(threadIdx.x & 63) + 512 * (threadIdx.x >> 6));
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t a = base + 8 * 128 * (it & 1);
        uint32_t x[16], y[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) rd<MODE>(a + 512 * (k & 3) + 128 * (k >> 2), x[k], y[k]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 16; ++k) acc += x[k] ^ y[k];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (threadIdx.x == 0) lds[0] = acc;
}

int main() {
    uint32_t *bad, *out;
    hipMalloc(&bad, 4);
    hipMalloc(&out, 4 * 256 * 4096);
    const char* names[6] = {"rd2  ", "b64  ", "b64u ", "rd2bc", "b64bc", "b32s2"};
    auto chk = [&](int m) {
        hipMemset(bad, 0, 4);
        switch (m) {
            case 0: hipLaunchKernelGGL(k_check<0>, dim3(1), dim3(256), 0, 0, bad); break;
            case 1: hipLaunchKernelGGL(k_check<1>, dim3(1), dim3(256), 0, 0, bad); break;
            case 2: hipLaunchKernelGGL(k_check<2>, dim3(1), dim3(256), 0, 0, bad); break;
            case 3: hipLaunchKernelGGL(k_check<3>, dim3(1), dim3(256), 0, 0, bad); break;
            case 4: hipLaunchKernelGGL(k_check<4>, dim3(1), dim3(256), 0, 0, bad); break;
            default: hipLaunchKernelGGL(k_check<5>, dim3(1), dim3(256), 0, 0, bad); break;
        }
        uint32_t h = 0;
        hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
        return h;
    };
    const int iters = 8192, blocks = 256 * 4;
    for (int m = 0; m < 6; ++m) {
        const uint32_t wrong = chk(m);
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            switch (m) {
                case 0: hipLaunchKernelGGL(k_time<0>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 1: hipLaunchKernelGGL(k_time<1>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 2: hipLaunchKernelGGL(k_time<2>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 3: hipLaunchKernelGGL(k_time<3>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 4: hipLaunchKernelGGL(k_time<4>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                default: hipLaunchKernelGGL(k_time<5>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        // CU-cycles per wave-instruction: 256 CUs, 2.4 GHz, blocks*4 waves, 16 reads per iteration
        const double winstr = blocks * 4.0 * iters * 16;
        printf("%s wrong lanes %3u/256: %.3f ms, %.2f CU-cycles per wave-instruction\n", names[m], wrong, best,
               best * 1e-3 * 2.4e9 * 256 / winstr);
    }
    return 0;
}

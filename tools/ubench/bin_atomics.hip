// k_bin's tile ranking in isolation (2^20 candidates on 2,400 tiles, 256
// workgroups of 1024 threads, 4 candidates per thread, an LDS histogram per
// workgroup): how the global phase's cost depends on the counter layout.
//   S = 1, 2, 4, 8, 16: one returning atomic per (workgroup, tile) on
//     counter[(b % S) * ntiles + tile] (S sub-counters per tile: S times
//     fewer workgroups on each counter's cache line), then the entry write
//   S = 0: no global atomic (the workgroup's histogram row is written): floor
// Each mode: 20 launches timed by HIP events (counters zeroed before each).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kBlock = 1024, kPer = 4, kMaxTiles = 4096;

__global__ __launch_bounds__(kBlock) void k_rank(const int* __restrict__ tile_of, int n, int ntiles, int S, int caps,
                                                 int* __restrict__ cnt, int2* __restrict__ out) {
    __shared__ int hist[kMaxTiles];
    for (int b = threadIdx.x; b < ntiles; b += kBlock) hist[b] = 0;
    __syncthreads();
    const int base = blockIdx.x * kBlock * kPer;
    int tl[kPer], lr[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        tl[k] = i < n ? tile_of[i] : -1;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        if (tl[k] >= 0) lr[k] = atomicAdd(&hist[tl[k]], 1);
    __syncthreads();
    const int s = S > 0 ? blockIdx.x % S : 0;
    int bs[kMaxTiles / kBlock];
#pragma unroll
    for (int j = 0; j < kMaxTiles / kBlock; ++j) {
        const int b = threadIdx.x + j * kBlock;
        const int c = b < ntiles ? hist[b] : 0;
        if (S > 0) bs[j] = c ? atomicAdd(&cnt[s * ntiles + b], c) : 0;
        else {
            if (b < ntiles) cnt[blockIdx.x * ntiles + b] = c;
            bs[j] = 0;
        }
    }
#pragma unroll
    for (int j = 0; j < kMaxTiles / kBlock; ++j) {
        const int b = threadIdx.x + j * kBlock;
        if (b < ntiles) hist[b] = bs[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        if (tl[k] < 0) continue;
        const int r = hist[tl[k]] + lr[k];
        if (r < caps) out[((long)tl[k] * (S > 0 ? S : 1) + s) * caps + r] = make_int2(i, tl[k]);
    }
}

int main() {
    const int n = 1 << 20, ntiles = 2400, nblk = (n + kBlock * kPer - 1) / (kBlock * kPer);
    std::vector<int> h(n);
    unsigned x = 12345u;
    for (int i = 0; i < n; ++i) {
        x = x * 1664525u + 1013904223u;
        h[i] = (int)((x >> 8) % ntiles);
    }
    int *d_tile, *d_cnt;
    int2* d_out;
    const int cap_total = 8192;
    if (hipMalloc(&d_tile, n * 4) || hipMalloc(&d_cnt, (size_t)nblk * ntiles * 4) ||
        hipMalloc(&d_out, (size_t)ntiles * cap_total * 8))
        return 1;
    (void)hipMemcpy(d_tile, h.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int S : {1, 2, 4, 8, 16, 0, 1, 8, 0}) {
        const int caps = cap_total / (S > 0 ? S : 1);
        float tot = 0.f;
        const int reps = 20;
        for (int r = 0; r < reps + 2; ++r) {
            (void)hipMemsetAsync(d_cnt, 0, (size_t)nblk * ntiles * 4, 0);
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_rank, dim3(nblk), dim3(kBlock), 0, 0, d_tile, n, ntiles, S, caps, d_cnt, d_out);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r >= 2) tot += ms;
        }
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        std::printf("S = %2d (%s): %7.2f us per launch\n", S, S > 0 ? "sub-counters" : "no global atomics",
                    tot / reps * 1e3f);
    }
    return 0;
}

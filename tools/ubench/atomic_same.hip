// How many returning atomics on ONE device counter a kernel can afford: each
// of W waves (lane 0) does one returning atomicAdd and stores the result, on
//   mode 0: one counter (all W on one address)
//   mode 1: W / 64 counters, 128 B apart (64 waves per counter)
//   mode 2: no atomic (the launch + store floor)
// W = 512 .. 65536 waves in workgroups of 256 threads; 20 launches each,
// timed by HIP events.  The question it answers: a pack or scorer that
// reserves output rows by one global atomic per wave / per item / per chunk.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_atom(int* __restrict__ cnt, int* __restrict__ out, int mode) {
    const int w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    if ((threadIdx.x & 63) != 0) return;
    int r = w;
    if (mode == 0) r = atomicAdd(cnt, 1);
    else if (mode == 1) r = atomicAdd(cnt + 32 * (w >> 6), 1);
    out[w] = r;
}

int main() {
    int *cnt, *out;
    const int maxw = 65536;
    if (hipMalloc(&cnt, sizeof(int) * 32 * (maxw / 64 + 1)) != hipSuccess) return 1;
    if (hipMalloc(&out, sizeof(int) * maxw) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int W = 512; W <= maxw; W *= 4) {
        for (int mode = 0; mode < 3; ++mode) {
            for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_atom, dim3(W / 4), dim3(256), 0, 0, cnt, out, mode);
            (void)hipEventRecord(e0, 0);
            for (int rep = 0; rep < 20; ++rep) hipLaunchKernelGGL(k_atom, dim3(W / 4), dim3(256), 0, 0, cnt, out, mode);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("waves %6d  mode %d (%s): %8.2f us per launch\n", W, mode,
                   mode == 0 ? "one counter" : mode == 1 ? "64 waves per counter" : "no atomic", ms / 20 * 1e3);
        }
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

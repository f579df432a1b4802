// k_bin's memory phases in isolation, to find which one sets its time
// (28 us per 2^20 candidates in the bench).  Same shapes as the bench: 2^20
// candidates with 3 binary64 coordinates and a reference view each, 2,400
// tiles with buckets of 6,992 entries (the engine's cap for this batch),
// 256 workgroups of 1024 threads, 4 candidates per thread.  The tile is a
// hash of the coordinates (the projection's arithmetic is not what is
// measured).  Phases switched by a bit mask:
//   1 the xy write (16 B per candidate), 2 the LDS histogram rank,
//   4 the returning global atomic per (workgroup, tile), 8 the bucket
//   scatter (8 B per candidate at tile * cap + rank),
//   16 the scatter staged: the workgroup's entries sorted by tile in LDS
//      first, so that each (workgroup, tile) run is written by adjacent lanes
// Each mode: 50 back-to-back launches between two events (counters zeroed by
// a memset inside the timed region, timed separately and subtracted).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kBlock = 1024, kPer = 4, kTiles = 2400, kCap = 6992, kLdsTiles = 4096;

__global__ __launch_bounds__(kBlock) void k_phases(const double* __restrict__ c, const int* __restrict__ ref, int n,
                                                   int mode, double* __restrict__ xy, int* __restrict__ cnt,
                                                   int2* __restrict__ out) {
    __shared__ int hist[kLdsTiles];
    __shared__ int2 stage[kBlock * kPer];
    __shared__ int scan_w[kBlock / 64 + 1];
    if (mode & 2)
        for (int b = threadIdx.x; b < kTiles; b += kBlock) hist[b] = 0;
    __syncthreads();
    const int base = blockIdx.x * kBlock * kPer;
    int tl[kPer], lr[kPer];
    double ck[kPer][3];
    int rk[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        const int ii = i < n ? i : 0;
        ck[k][0] = c[3 * ii];
        ck[k][1] = c[3 * ii + 1];
        ck[k][2] = c[3 * ii + 2];
        rk[k] = ref[ii];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        tl[k] = -1;
        lr[k] = 0;
        if (i >= n) continue;
        const double px = ck[k][0] * 640.0, py = ck[k][1] * 480.0 + 1e-9 * ck[k][2];
        if (mode & 1) {
            xy[2 * i] = px;
            xy[2 * i + 1] = py;
        }
        const int tx = min(max((int)px, 0), 639) / 16, ty = min(max((int)py, 0), 479) / 8;
        tl[k] = (ty * 40 + tx + rk[k]) % kTiles;
        if (mode & 2) lr[k] = atomicAdd(&hist[tl[k]], 1);
    }
    __syncthreads();
    if (mode & 4) {
        int bs[kLdsTiles / kBlock];
#pragma unroll
        for (int j = 0; j < kLdsTiles / kBlock; ++j) {
            const int b = threadIdx.x + j * kBlock;
            const int h = b < kTiles ? hist[b] : 0;
            bs[j] = h ? atomicAdd(&cnt[b], h) : 0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kLdsTiles / kBlock; ++j) {
            const int b = threadIdx.x + j * kBlock;
            if (b < kTiles) hist[b] = bs[j] | (b < kTiles ? 0 : 0);
        }
        __syncthreads();
    }
    if (mode & 16) {
        // local exclusive scan of the histogram -> local offsets; entries
        // written to LDS in tile order, then each lane writes one entry
        // (adjacent lanes: the same tile's run, consecutive addresses)
        __shared__ int loc[kLdsTiles];
        __shared__ int gb[kLdsTiles];
        // the histogram's counts again (the global phase overwrote hist with bases)
        for (int b = threadIdx.x; b < kTiles; b += kBlock) loc[b] = 0;
        __syncthreads();
        int lr2[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) lr2[k] = tl[k] >= 0 ? atomicAdd(&loc[tl[k]], 1) : 0;
        __syncthreads();
        // scan loc (kTiles <= 4 per thread)
        int v[kLdsTiles / kBlock], s = 0;
#pragma unroll
        for (int j = 0; j < kLdsTiles / kBlock; ++j) {
            const int b = threadIdx.x * (kLdsTiles / kBlock) + j;
            v[j] = b < kTiles ? loc[b] : 0;
            s += v[j];
        }
        int incl = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(incl, d, 64);
            if ((threadIdx.x & 63) >= d) incl += o;
        }
        if ((threadIdx.x & 63) == 63) scan_w[threadIdx.x >> 6] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            int run = 0;
            for (int w = 0; w < kBlock / 64; ++w) { const int t = scan_w[w]; scan_w[w] = run; run += t; }
        }
        __syncthreads();
        int ex = scan_w[threadIdx.x >> 6] + incl - s;
#pragma unroll
        for (int j = 0; j < kLdsTiles / kBlock; ++j) {
            const int b = threadIdx.x * (kLdsTiles / kBlock) + j;
            if (b < kTiles) {
                gb[b] = ex;   // local start of tile b's run
                ex += v[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = base + k * kBlock + threadIdx.x;
            if (tl[k] >= 0) stage[gb[tl[k]] + lr2[k]] = make_int2(i, tl[k]);
        }
        __syncthreads();
        const int tot = min(n - base, kBlock * kPer);
        for (int e = threadIdx.x; e < tot; e += kBlock) {
            const int2 en = stage[e];
            const int t = en.y;
            const int r = ((mode & 4) ? hist[t] : 0) + (e - gb[t]);
            if (r < kCap) out[(long)t * kCap + r] = en;
        }
        return;
    }
    if (mode & 8) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int i = base + k * kBlock + threadIdx.x;
            if (tl[k] < 0) continue;
            const int r = ((mode & 4) ? hist[tl[k]] : 0) + lr[k];
            if (r < kCap) out[(long)tl[k] * kCap + r] = make_int2(i, tl[k]);
        }
    }
}

// The atomic-free alternative in three launches: (1) project, LDS rank,
// the workgroup's histogram row written out, each candidate's (tile, local
// rank) kept in a scratch word; (2) per tile, the exclusive prefix of its
// column over the workgroups (+ the tile's total); (3) the scatter.
__global__ __launch_bounds__(kBlock) void k_count(const double* __restrict__ c, const int* __restrict__ ref, int n,
                                                  double* __restrict__ xy, int* __restrict__ rows,
                                                  int2* __restrict__ scratch) {
    __shared__ int hist[kLdsTiles];
    for (int b = threadIdx.x; b < kTiles; b += kBlock) hist[b] = 0;
    __syncthreads();
    const int base = blockIdx.x * kBlock * kPer;
    int tl[kPer], lr[kPer];
    double ck[kPer][3];
    int rk[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        const int ii = i < n ? i : 0;
        ck[k][0] = c[3 * ii];
        ck[k][1] = c[3 * ii + 1];
        ck[k][2] = c[3 * ii + 2];
        rk[k] = ref[ii];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        tl[k] = -1;
        if (i >= n) continue;
        const double px = ck[k][0] * 640.0, py = ck[k][1] * 480.0 + 1e-9 * ck[k][2];
        xy[2 * i] = px;
        xy[2 * i + 1] = py;
        const int tx = min(max((int)px, 0), 639) / 16, ty = min(max((int)py, 0), 479) / 8;
        tl[k] = (ty * 40 + tx + rk[k]) % kTiles;
        lr[k] = atomicAdd(&hist[tl[k]], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kTiles; b += kBlock) rows[(long)blockIdx.x * kTiles + b] = hist[b];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        if (i < n) scratch[i] = make_int2(tl[k], lr[k]);
    }
}

// tile columns: 64 tiles x 16 segments of nblk / 16 workgroups per block
__global__ __launch_bounds__(1024) void k_colscan(int nblk, int* __restrict__ rows, int* __restrict__ cnt) {
    __shared__ int seg[16][65];
    const int tl = threadIdx.x & 63, sg = threadIdx.x >> 6;
    const int tile = blockIdx.x * 64 + tl;
    const int per = nblk / 16;
    int v[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int w = sg * per + k;
        v[k] = (tile < kTiles && k < per) ? rows[(long)w * kTiles + tile] : 0;
        s += v[k];
    }
    seg[sg][tl] = s;
    __syncthreads();
    int pre = 0;
    for (int q = 0; q < sg; ++q) pre += seg[q][tl];
    if (sg == 15 && tile < kTiles) cnt[tile] = pre + s;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int w = sg * per + k;
        if (tile < kTiles && k < per) rows[(long)w * kTiles + tile] = pre;
        pre += v[k];
    }
}

__global__ __launch_bounds__(kBlock) void k_scatter(int n, const int* __restrict__ rows, const int2* __restrict__ scratch,
                                                    int2* __restrict__ out) {
    const int base = blockIdx.x * kBlock * kPer;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = base + k * kBlock + threadIdx.x;
        if (i >= n) continue;
        const int2 s = scratch[i];
        const int r = rows[(long)blockIdx.x * kTiles + s.x] + s.y;
        if (r < kCap) out[(long)s.x * kCap + r] = make_int2(i, s.x);
    }
}

int main() {
    const int n = 1 << 20, nblk = n / (kBlock * kPer);
    std::vector<double> hc(3 * (size_t)n);
    std::vector<int> hr(n);
    unsigned x = 12345u;
    auto rnd = [&]() {
        x = x * 1664525u + 1013904223u;
        return (double)(x >> 8) / 16777216.0;
    };
    for (int i = 0; i < n; ++i) {
        hc[3 * i] = rnd();
        hc[3 * i + 1] = rnd();
        hc[3 * i + 2] = rnd();
        hr[i] = (int)(rnd() * 48);
    }
    double *d_c, *d_xy;
    int *d_ref, *d_cnt;
    int2* d_out;
    if (hipMalloc(&d_c, 24 * (size_t)n) || hipMalloc(&d_ref, 4 * (size_t)n) || hipMalloc(&d_xy, 16 * (size_t)n) ||
        hipMalloc(&d_cnt, 4 * kTiles) || hipMalloc(&d_out, (size_t)kTiles * kCap * 8))
        return 1;
    (void)hipMemcpy(d_c, hc.data(), 24 * (size_t)n, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ref, hr.data(), 4 * (size_t)n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 50;
    auto timeit = [&](int mode, bool launch) {
        float best = 1e30f;
        for (int trial = 0; trial < 3; ++trial) {
            (void)hipEventRecord(e0, 0);
            for (int r = 0; r < reps; ++r) {
                (void)hipMemsetAsync(d_cnt, 0, 4 * kTiles, 0);
                if (launch) hipLaunchKernelGGL(k_phases, dim3(nblk), dim3(kBlock), 0, 0, d_c, d_ref, n, mode, d_xy, d_cnt, d_out);
            }
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        return best / reps * 1e3f;
    };
    const float memset_us = timeit(0, false);
    std::printf("memset alone: %.2f us\n", memset_us);
    struct M { int mode; const char* what; };
    for (M m : {M{0, "loads only"}, M{1, "+ xy write"}, M{2, "+ LDS rank"}, M{3, "xy + LDS rank"},
                M{6, "LDS rank + global atomics"}, M{10, "LDS rank + scatter (no atomics)"},
                M{14, "LDS rank + atomics + scatter"}, M{15, "all (k_bin's shape)"},
                M{2 | 4 | 16, "LDS rank + atomics + staged scatter"}, M{1 | 2 | 4 | 16, "all, staged scatter"},
                M{15, "all (again)"}}) {
        const float us = timeit(m.mode, true) - memset_us;
        std::printf("mode %2d %-40s %7.2f us per launch\n", m.mode, m.what, us);
    }
    {
        int* d_rows;
        int2* d_scr;
        if (hipMalloc(&d_rows, (size_t)nblk * kTiles * 4) || hipMalloc(&d_scr, 8 * (size_t)n)) return 1;
        float best = 1e30f;
        for (int trial = 0; trial < 3; ++trial) {
            (void)hipEventRecord(e0, 0);
            for (int r = 0; r < reps; ++r) {
                (void)hipMemsetAsync(d_cnt, 0, 4 * kTiles, 0);
                hipLaunchKernelGGL(k_count, dim3(nblk), dim3(kBlock), 0, 0, d_c, d_ref, n, d_xy, d_rows, d_scr);
                hipLaunchKernelGGL(k_colscan, dim3((kTiles + 63) / 64), dim3(1024), 0, 0, nblk, d_rows, d_cnt);
                hipLaunchKernelGGL(k_scatter, dim3(nblk), dim3(kBlock), 0, 0, n, d_rows, d_scr, d_out);
            }
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        std::printf("three launches: count + column scan + scatter (no global atomics) %7.2f us per batch\n",
                    best / reps * 1e3f - memset_us);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}

// Accuracy of w = 1/sqrt(D) for the scorer's table (k_score_mma phase 2):
// v_rsq_f64 alone, + 1 and + 2 Newton steps, against the correctly rounded
// 1/sqrt in long double on the host.  D = n S_bb - S_b^2 < 2^31.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void k(const double* D, double* w0, double* w1, double* w2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = D[i];
    double y = __builtin_amdgcn_rsq(d);
    w0[i] = y;
    y = y * (1.5 - 0.5 * d * y * y);
    w1[i] = y;
    y = y * (1.5 - 0.5 * d * y * y);
    w2[i] = y;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> D(n), w0(n), w1(n), w2(n);
    std::mt19937_64 g(1);
    for (int i = 0; i < n; ++i) D[i] = (double)(1 + g() % ((1ull << 31) - 1));
    for (int i = 0; i < 64; ++i) D[i] = (double)(i + 1);
    double *dD, *d0, *d1, *d2;
    hipMalloc(&dD, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8);
    hipMemcpy(dD, D.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dD, d0, d1, d2, n);
    hipMemcpy(w0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(w1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(w2.data(), d2, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double r = 1.0L / sqrtl((long double)D[i]);
        e0 = std::fmax(e0, (double)fabsl((w0[i] - r) / r));
        e1 = std::fmax(e1, (double)fabsl((w1[i] - r) / r));
        e2 = std::fmax(e2, (double)fabsl((w2[i] - r) / r));
    }
    printf("max relative error over %d values: rsq %.3e, +1 Newton %.3e, +2 Newton %.3e\n", n, e0, e1, e2);
    return 0;
}

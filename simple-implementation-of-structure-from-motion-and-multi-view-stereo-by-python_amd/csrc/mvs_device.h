// Device helpers shared by the HIP translation units (mvs_kernels.hip,
// sfm_kernels.hip): the reference's projection, window bounds and ctNcc in
// numpy's operation order.  Compiled with -ffp-contract=off: every fused
// product is written as fma() (numpy/OpenBLAS 3-element dot products).
#pragma once
#include "mvs_internal.h"

#define DEV __device__ __forceinline__

namespace {

// |ncc - thr| band (absolute) inside which a closed-form value is replaced by
// the numpy-order ctNcc before the decision
constexpr double kGuard = 1e-9;

// Python int() of a float64 pixel coordinate (truncation toward zero).  The
// reference raises on nan/inf; here such a point is simply not valid.
DEV bool py_trunc(double v, int* out) {
    if (!(v > -1e9 && v < 1e9)) return false;
    *out = (int)v;
    return true;
}

// cv2.projectPoints with zero distortion (cvProjectPoints2Internal order).
DEV void project(const CamDev& cm, const double* c, double& px, double& py) {
    const double X = c[0], Y = c[1], Z = c[2];
    double x = cm.Rp[0] * X + cm.Rp[1] * Y + cm.Rp[2] * Z + cm.t[0];
    double y = cm.Rp[3] * X + cm.Rp[4] * Y + cm.Rp[5] * Z + cm.t[1];
    double z = cm.Rp[6] * X + cm.Rp[7] * Y + cm.Rp[8] * Z + cm.t[2];
    z = z != 0.0 ? 1.0 / z : 1.0;
    x *= z;
    y *= z;
    px = x * cm.fx + cm.cx;
    py = y * cm.fy + cm.cy;
}

// The same projection from 16 values [R' (9), t (3), fx, fy, cx, cy], value
// k = cv(k) (k_bin keeps them in LDS, field-major); identical operations in
// the same order.
template <class CV>
DEV void project_vals(CV&& cv, const double* c, double& px, double& py) {
    const double X = c[0], Y = c[1], Z = c[2];
    double x = cv(0) * X + cv(1) * Y + cv(2) * Z + cv(9);
    double y = cv(3) * X + cv(4) * Y + cv(5) * Z + cv(10);
    double z = cv(6) * X + cv(7) * Y + cv(8) * Z + cv(11);
    z = z != 0.0 ? 1.0 / z : 1.0;
    x *= z;
    y *= z;
    px = x * cv(12) + cv(14);
    py = y * cv(13) + cv(15);
}

// getDescFeatures bounds (HarrisFeatures.py:128), row = y, col = x.
DEV bool window_ok(const SceneDev& sc, double px, double py, int wid, int* q, int* r) {
    int rr, qq;
    if (!py_trunc(py, &rr) || !py_trunc(px, &qq)) return false;
    if (!(rr - wid >= 0 && rr + wid + 1 < sc.H && qq - wid > 0 && qq + wid + 1 < sc.W)) return false;
    *q = qq;
    *r = rr;
    return true;
}

// numpy pairwise sum of (x_i - mean)^2 for n <= 128 (8 accumulators).
template <class F>
DEV double pairwise_sq(F&& xi, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; i++) { double x = xi(i); res += x * x; }
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) { double x = xi(j); r[j] = x * x; }
    int i;
    for (i = 8; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) { double x = xi(i + j); r[j] += x * x; }
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) { double x = xi(i); res += x * x; }
    return res;
}

// ctNcc (MVS2.py:39-43) in numpy's operation order; A(i), B(i) return pixel i.
template <class FA, class FB>
DEV double exact_ncc_generic(FA&& A, FB&& B, int n) {
    int64_t sa = 0, sb = 0;
    for (int i = 0; i < n; i++) { sa += A(i); sb += B(i); }
    const double ma = (double)sa / n, mb = (double)sb / n;
    const double stda = sqrt(pairwise_sq([&](int i) { return (double)A(i) - ma; }, n) / n);
    const double stdb = sqrt(pairwise_sq([&](int i) { return (double)B(i) - mb; }, n) / n);
    double s = 0;
    for (int i = 0; i < n; i++) s = s + (((double)A(i) - ma) / stda) * (((double)B(i) - mb) / stdb);
    return s / (n - 1);
}

// ctNcc in numpy's order with the pixel count known at compile time: every
// loop unrolls, so pixel i's byte comes from a register (constant index).
template <int N, class FA, class FB>
DEV double exact_ncc_fixed(FA&& A, FB&& B) {
    int sa = 0, sb = 0;
#pragma unroll
    for (int i = 0; i < N; i++) { sa += A(i); sb += B(i); }
    const double ma = (double)sa / N, mb = (double)sb / N;
    auto pairwise = [&](auto&& X, double m) {
        // numpy pairwise sum of (x - m)^2 for N <= 128: 8 accumulators
        if constexpr (N < 8) {
            double res = 0.;
#pragma unroll
            for (int i = 0; i < N; i++) { const double x = X(i) - m; res += x * x; }
            return res;
        } else {
            double acc[8];
#pragma unroll
            for (int j = 0; j < 8; j++) { const double x = X(j) - m; acc[j] = x * x; }
#pragma unroll
            for (int i = 8; i < N - (N % 8); i += 8)
#pragma unroll
                for (int j = 0; j < 8; j++) { const double x = X(i + j) - m; acc[j] += x * x; }
            double res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
#pragma unroll
            for (int i = N - (N % 8); i < N; i++) { const double x = X(i) - m; res += x * x; }
            return res;
        }
    };
    static_assert(N <= 128, "numpy pairwise summation restated for n <= 128");
    const double stda = sqrt(pairwise([&](int i) { return (double)A(i); }, ma) / N);
    const double stdb = sqrt(pairwise([&](int i) { return (double)B(i); }, mb) / N);
    double s = 0;
#pragma unroll
    for (int i = 0; i < N; i++) s = s + (((double)A(i) - ma) / stda) * (((double)B(i) - mb) / stdb);
    return s / (N - 1);
}

}  // namespace

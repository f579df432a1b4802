// HIP kernels for the MVS2 photo-consistency hot path (gfx950 / CDNA4).
//
// Reference path (MarvinChung/simple-implementation-of-structure-from-motion-
// and-multi-view-stereo-by-python):
//   MyPatch.photo_consistenecy_test   MVS2.py:62-77   -> wave_score<>
//   projectPoint                      utils.py:241-244 -> project()
//   getDescFeatures                   HarrisFeatures.py:116-133 -> window gather
//   ctNcc                             MVS2.py:39-43   -> integer moments + exact_ncc<>
//   patch_expansion candidate geometry + accept test MVS2.py:329-369 -> k_expand
//
// Numerics.  Window sums are exact integers (S_a, S_aa, S_b, S_bb, S_ab); the
// NCC is evaluated in closed form  ncc = n*(n*S_ab - S_a*S_b) /
// ((n-1)*sqrt((n*S_aa - S_a^2)(n*S_bb - S_b^2))).  When that value lies within
// 1e-9 of the threshold the lane recomputes ctNcc in numpy's exact operation
// order (exact_ncc), so every accept/reject decision is the reference's.
// Geometry is binary64 in the reference's order; this file must be compiled
// with -ffp-contract=off (products that numpy/OpenBLAS fuse are written as
// fma() explicitly).
#include "mvs_internal.h"

#define DEV __device__ __forceinline__

namespace {

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

// getDescFeatures bounds (HarrisFeatures.py:128), row = y, col = x.
DEV bool window_ok(const SceneDev& sc, double px, double py, int wid, int* q, int* r) {
    int rr, qq;
    if (!py_trunc(py, &rr) || !py_trunc(px, &qq)) return false;
    if (!(rr - wid >= 0 && rr + wid + 1 < sc.H && qq - wid > 0 && qq + wid + 1 < sc.W)) return false;
    *q = qq;
    *r = rr;
    return true;
}

DEV uint8_t stack_px(const SceneDev& sc, int view, int y, int x) {
    return sc.stack[(int64_t)y * sc.row_bytes + (int64_t)(x >> 2) * sc.V * 4 + view * 4 + (x & 3)];
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

template <int WID>
__device__ __noinline__ double exact_ncc_stack(const SceneDev sc, int R, int v, int q, int r) {
    constexpr int NB = 2 * WID + 1;
    auto A = [&](int i) -> int { return stack_px(sc, R, r - WID + i / NB, q - WID + i % NB); };
    auto B = [&](int i) -> int { return stack_px(sc, v, r - WID + i / NB, q - WID + i % NB); };
    return exact_ncc_generic(A, B, NB * NB);
}

DEV double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// One wave scores one candidate whose window sits at (q, r) of every view
// (the reference samples all views at view R's pixel, MVS2.py:68).
// Lane l handles views l, l+64, ... (NS slots).  Returns nothing; lane 0 of
// the wave writes mask/count/avg.
template <int WID, int NS>
DEV void wave_score(const SceneDev& sc, int R, int q, int r, double thr, uint64_t* mask_out,
                    int32_t* count_out, double* avg_out, int32_t* exact_hits) {
    constexpr int NB = 2 * WID + 1;
    constexpr int NPX = NB * NB;
    constexpr int NW = (NB + 3) / 4;
    constexpr int ND = NW + 1;
    constexpr uint32_t LASTMASK = (NB % 4 == 0) ? 0xffffffffu : ((1u << (8 * (NB % 4))) - 1u);
    const int lane = threadIdx.x & 63;
    const int q0 = q - WID;
    const int k0 = q0 >> 2, o = q0 & 3;
    const int V = sc.V;
    const int64_t vstride = (int64_t)V * 4;
    const uint8_t* p0 = sc.stack + (int64_t)(r - WID) * sc.row_bytes + (int64_t)k0 * vstride;
    const int Rs = R >> 6, Rl = R & 63;

    uint32_t Sb[NS], Sbb[NS], Sab[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) Sb[s] = Sbb[s] = Sab[s] = 0;

    for (int row = 0; row < NB; ++row) {
        const uint8_t* prow = p0 + (int64_t)row * sc.row_bytes;
        uint32_t w[NS][NW];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int v = lane + 64 * s;
            uint32_t d[ND];
            if (v < V) {
                const uint8_t* pv = prow + v * 4;
#pragma unroll
                for (int j = 0; j < ND; ++j) d[j] = *(const uint32_t*)(pv + j * vstride);
            } else {
#pragma unroll
                for (int j = 0; j < ND; ++j) d[j] = 0;
            }
#pragma unroll
            for (int j = 0; j < NW; ++j) w[s][j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], o);
            w[s][NW - 1] &= LASTMASK;
        }
        uint32_t a[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            uint32_t src = w[0][j];
#pragma unroll
            for (int s = 1; s < NS; ++s) src = (Rs == s) ? w[s][j] : src;
            a[j] = __builtin_amdgcn_readlane(src, Rl);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                Sab[s] = __builtin_amdgcn_udot4(a[j], w[s][j], Sab[s], false);
                Sbb[s] = __builtin_amdgcn_udot4(w[s][j], w[s][j], Sbb[s], false);
                Sb[s] = __builtin_amdgcn_sad_u8(w[s][j], 0u, Sb[s]);
            }
        }
    }

    uint32_t sa_src = Sb[0], saa_src = Sbb[0];
#pragma unroll
    for (int s = 1; s < NS; ++s) {
        sa_src = (Rs == s) ? Sb[s] : sa_src;
        saa_src = (Rs == s) ? Sbb[s] : saa_src;
    }
    const int64_t Sa = __builtin_amdgcn_readlane(sa_src, Rl);
    const int64_t Saa = __builtin_amdgcn_readlane(saa_src, Rl);
    const int64_t da = (int64_t)NPX * Saa - Sa * Sa;

    double acc = 0.0;
    int cnt = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int v = lane + 64 * s;
        const int64_t sb = Sb[s];
        const int64_t db = (int64_t)NPX * (int64_t)Sbb[s] - sb * sb;
        const int64_t num = (int64_t)NPX * (int64_t)Sab[s] - Sa * sb;
        bool pass = false;
        double ncc = 0.0;
        if (v < V && v != R && da > 0 && db > 0) {   // da or db == 0: ctNcc is nan -> rejected
            ncc = (double)((int64_t)NPX * num) /
                  ((double)(NPX - 1) * sqrt((double)da * (double)db));
            if (fabs(ncc - thr) <= kGuard) {
                ncc = exact_ncc_stack<WID>(sc, R, v, q, r);
                atomicAdd(exact_hits, 1);
            }
            pass = ncc > thr;
        }
        const uint64_t m = __ballot(pass);
        if (lane == 0) mask_out[s] = m;
        cnt += __popcll(m);
        acc += pass ? ncc : 0.0;
    }
    const double tot = wave_sum(acc);
    if (lane == 0) {
        *count_out = cnt;
        if (avg_out) *avg_out = cnt > 0 ? tot / cnt : 0.0;
    }
}

template <int NS>
DEV void wave_score_empty(uint64_t* mask_out, int32_t* count_out, double* avg_out) {
    const int lane = threadIdx.x & 63;
    if (lane < NS) mask_out[lane] = 0;
    if (lane == 0) {
        *count_out = 0;
        if (avg_out) *avg_out = 0.0;
    }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// RGB (V,H,W,3) -> gray stack[y][k][v][4]; gray = OpenCV BGR2GRAY applied to
// RGB data (HarrisFeatures.py:125 on main.py:18's RGB images).
__global__ void k_build_stack(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ stack, int V,
                              int H, int W, int Wq) {
    const int64_t total = (int64_t)H * Wq * V;
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int v = (int)(id % V);
        const int64_t yk = id / V;
        const int k = (int)(yk % Wq), y = (int)(yk / Wq);
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int x = 4 * k + b;
            uint32_t g = 0;
            if (x < W) {
                const uint8_t* p = rgb + (((int64_t)v * H + y) * W + x) * 3;
                g = (p[0] * 1868u + p[1] * 9617u + p[2] * 4899u + 8192u) >> 14;
            }
            word |= g << (8 * b);
        }
        *(uint32_t*)(stack + (int64_t)y * Wq * V * 4 + (int64_t)k * V * 4 + v * 4) = word;
    }
}

template <int WID, int NS>
__global__ __launch_bounds__(256) void k_score(const SceneDev sc, const ScoreArgs a) {
    const int64_t cand = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (cand >= a.n) return;
    const int words = (sc.V + 63) >> 6;
    const int R = __builtin_amdgcn_readfirstlane(a.ref[cand]);
    double c[3] = {a.c[3 * cand], a.c[3 * cand + 1], a.c[3 * cand + 2]};
    double px, py;
    project(sc.cams[R], c, px, py);
    const int lane = threadIdx.x & 63;
    if (lane == 0) { a.xy[2 * cand] = px; a.xy[2 * cand + 1] = py; }
    int q, r;
    if (!window_ok(sc, px, py, WID, &q, &r)) {
        wave_score_empty<NS>(a.mask + cand * words, a.count + cand, a.avg + cand);
        return;
    }
    q = __builtin_amdgcn_readfirstlane(q);
    r = __builtin_amdgcn_readfirstlane(r);
    wave_score<WID, NS>(sc, R, q, r, a.thr, a.mask + cand * words, a.count + cand, a.avg + cand,
                        a.exact_hits);
}

DEV double dot3(const double* a, const double* b) {
    // np.dot of two float64 3-vectors as OpenBLAS 0.3.29 evaluates it.
    return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]));
}

DEV int py_wrap(int i, int n) { return i < 0 ? i + n : i; }

// patch_expansion candidate (MVS2.py:329-369): one wave per child.
template <int WID, int NS>
__global__ __launch_bounds__(256) void k_expand(const SceneDev sc, RecordsDev rec,
                                                 const ExpandArgs a) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= a.n) return;
    const int lane = threadIdx.x & 63;
    const int words = (sc.V + 63) >> 6;
    const ChildJob job = a.jobs[k];
    const int64_t par = job.parent;
    const int v = __builtin_amdgcn_readfirstlane((int)job.view);
    const int di = job.di;
    const int64_t out = a.first_out + k;
    const CamDev& cm = sc.cams[v];
    const double pc[3] = {rec.c[3 * par], rec.c[3 * par + 1], rec.c[3 * par + 2]};
    const double pn[3] = {rec.n[3 * par], rec.n[3 * par + 1], rec.n[3 * par + 2]};
    const double cs = (double)a.cell_size;
    // which_cell of the parent's hit (MVS2.py:330): every V entry carries the
    // parent's projection into its own reference view (MVS2.py:68, 74).
    const double ci = floor(rec.xy[2 * par] / cs), cj = floor(rec.xy[2 * par + 1] / cs);
    // cell_center(ci+i, cj+i): the second index reuses i (MVS2.py:334)
    const double cc0 = cs * ((ci + di) + 0.5);
    const double cc1 = cs * ((cj + di) + 0.5);
    const double w[3] = {cc0 - cm.cx, cc1 - cm.cy, cm.fbar};
    double Pw[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)   // R^T @ w + C (MVS2.py:353)
        Pw[j] = fma(cm.R[6 + j], w[2], fma(cm.R[3 + j], w[1], cm.R[j] * w[0])) + cm.C[j];
    const double nrm = sqrt((Pw[0] * Pw[0] + Pw[1] * Pw[1]) + Pw[2] * Pw[2]);   // vector_norm
    const double d[3] = {Pw[0] / nrm, Pw[1] / nrm, Pw[2] / nrm};
    // ray_plane_intersection(camera_pos[v], d, parent.c, parent.n) (MVS2.py:302-306)
    const double dot_out = dot3(d, pn);
    const double cmo[3] = {pc[0] - cm.O[0], pc[1] - cm.O[1], pc[2] - cm.O[2]};
    const double tt = dot3(cmo, pn) / dot_out;
    double X[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) X[j] = cm.O[j] + tt * d[j];
    const double e0 = X[0] - cm.O[0], e1 = X[1] - cm.O[1], e2 = X[2] - cm.O[2];
    const double dist = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
    double nX[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) nX[j] = (cm.O[j] - X[j]) / dist;

    double px, py;
    project(cm, X, px, py);
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) { rec.c[3 * out + j] = X[j]; rec.n[3 * out + j] = nX[j]; }
        rec.xy[2 * out] = px;
        rec.xy[2 * out + 1] = py;
        rec.R[out] = v;
        // get_color(imgs[v], cc0, cc1) = img[int(cc1)][int(cc0)] (MVS2.py:119-120, 358)
        int yy = 0, xx = 0;
        py_trunc(cc1, &yy);
        py_trunc(cc0, &xx);
        yy = py_wrap(yy, sc.H);
        xx = py_wrap(xx, sc.W);
        uint8_t rgbv[3] = {0, 0, 0};
        if (yy >= 0 && yy < sc.H && xx >= 0 && xx < sc.W) {
            const uint8_t* p = sc.rgb + (((int64_t)v * sc.H + yy) * sc.W + xx) * 3;
            rgbv[0] = p[0]; rgbv[1] = p[1]; rgbv[2] = p[2];
        }
        rec.color[4 * out] = rgbv[0]; rec.color[4 * out + 1] = rgbv[1];
        rec.color[4 * out + 2] = rgbv[2]; rec.color[4 * out + 3] = 0;
        rec.cell[2 * out] = (int32_t)floor(px / cs);
        rec.cell[2 * out + 1] = (int32_t)floor(py / cs);
    }
    int q, r;
    if (!window_ok(sc, px, py, WID, &q, &r)) {
        wave_score_empty<NS>(rec.mask + out * words, rec.count + out, nullptr);
        if (lane == 0) rec.accept[out] = 0;
        return;
    }
    q = __builtin_amdgcn_readfirstlane(q);
    r = __builtin_amdgcn_readfirstlane(r);
    wave_score<WID, NS>(sc, v, q, r, a.thr, rec.mask + out * words, rec.count + out, nullptr,
                        a.exact_hits);
    if (lane == 0) {
        // accept test (MVS2.py:369) with is_patch_neighbor (MVS2.py:298-299)
        const double pm[3] = {pc[0] - X[0], pc[1] - X[1], pc[2] - X[2]};
        const double nb = fabs(dot3(pm, pn) + dot3(pm, nX));
        const double g0 = pc[0] - X[0], g1 = pc[1] - X[1], g2 = pc[2] - X[2];
        const double dd = sqrt((g0 * g0 + g1 * g1) + g2 * g2);
        const int cnt = rec.count[out];
        rec.accept[out] = (cnt >= a.vlb && nb < 0.1 && dd < a.dist_thr) ? 1 : 0;
    }
}

// Batched ctNcc on explicit window pairs: the function-level check of the NCC
// core (integer moments + guard + exact fallback), one thread per pair.
__global__ void k_ncc_windows(int64_t n, int npx, const uint8_t* __restrict__ A,
                              const uint8_t* __restrict__ B, double thr, int force_exact,
                              double* ncc_out, uint8_t* pass_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t* a = A + i * npx;
        const uint8_t* b = B + i * npx;
        int64_t sa = 0, sb = 0, saa = 0, sbb = 0, sab = 0;
        for (int k = 0; k < npx; ++k) {
            const int x = a[k], y = b[k];
            sa += x; sb += y; saa += x * x; sbb += y * y; sab += x * y;
        }
        const int64_t da = npx * saa - sa * sa, db = npx * sbb - sb * sb;
        const int64_t num = npx * sab - sa * sb;
        double ncc;
        bool in_guard = false;
        if (da <= 0 || db <= 0) {
            ncc = __builtin_nan("");
        } else {
            ncc = (double)(npx * num) / ((double)(npx - 1) * sqrt((double)da * (double)db));
            in_guard = fabs(ncc - thr) <= kGuard;
        }
        if ((force_exact || in_guard) && da > 0 && db > 0)
            ncc = exact_ncc_generic([&](int k) -> int { return a[k]; },
                                    [&](int k) -> int { return b[k]; }, npx);
        ncc_out[i] = ncc;
        pass_out[i] = ncc > thr ? 1 : 0;
    }
}

template <int WID>
int launch_score_w(const SceneDev* sc, const ScoreArgs* a, hipStream_t s) {
    const int64_t blocks = (a->n + 3) / 4;
    if (blocks == 0) return 0;
    if (sc->V <= 64)
        hipLaunchKernelGGL((k_score<WID, 1>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, *a);
    else if (sc->V <= 128)
        hipLaunchKernelGGL((k_score<WID, 2>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, *a);
    else
        hipLaunchKernelGGL((k_score<WID, 4>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, *a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int WID>
int launch_expand_w(const SceneDev* sc, RecordsDev rec, const ExpandArgs* a, hipStream_t s) {
    const int64_t blocks = (a->n + 3) / 4;
    if (blocks == 0) return 0;
    if (sc->V <= 64)
        hipLaunchKernelGGL((k_expand<WID, 1>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, rec, *a);
    else if (sc->V <= 128)
        hipLaunchKernelGGL((k_expand<WID, 2>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, rec, *a);
    else
        hipLaunchKernelGGL((k_expand<WID, 4>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, rec, *a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

extern "C" int mvs_launch_build_stack(const uint8_t* d_rgb, uint8_t* d_stack, int V, int H, int W,
                                      int Wq, hipStream_t s) {
    const int64_t total = (int64_t)H * Wq * V;
    const int blocks = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
    hipLaunchKernelGGL(k_build_stack, dim3(blocks), dim3(256), 0, s, d_rgb, d_stack, V, H, W, Wq);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_score(const SceneDev* sc, const ScoreArgs* a, int wid, hipStream_t s) {
    switch (wid) {
        case 1: return launch_score_w<1>(sc, a, s);
        case 2: return launch_score_w<2>(sc, a, s);
        case 3: return launch_score_w<3>(sc, a, s);
        case 4: return launch_score_w<4>(sc, a, s);
        case 5: return launch_score_w<5>(sc, a, s);
        default: return -2;
    }
}

extern "C" int mvs_launch_expand(const SceneDev* sc, RecordsDev rec, const ExpandArgs* a, int wid,
                                 hipStream_t s) {
    switch (wid) {
        case 3: return launch_expand_w<3>(sc, rec, a, s);
        case 5: return launch_expand_w<5>(sc, rec, a, s);
        default: return -2;
    }
}

extern "C" int mvs_launch_ncc_windows(int64_t n, int npx, const uint8_t* a, const uint8_t* b,
                                      double thr, int force_exact, double* ncc, uint8_t* pass,
                                      hipStream_t s) {
    if (npx <= 0 || npx > 128) return -2;
    const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_ncc_windows, dim3(blocks), dim3(256), 0, s, n, npx, a, b, thr, force_exact,
                       ncc, pass);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

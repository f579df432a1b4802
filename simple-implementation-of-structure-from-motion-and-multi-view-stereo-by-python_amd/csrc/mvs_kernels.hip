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
#include <algorithm>
#include <cstdlib>

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

// One 12-byte moments entry as three dword loads (4-byte aligned).
DEV MomEntry load_mom(const MomEntry* m, int64_t idx) {
    const uint32_t* p = (const uint32_t*)m + 3 * idx;
    MomEntry e;
    e.w = __longlong_as_double(((unsigned long long)p[1] << 32) | p[0]);
    e.sb = p[2];
    return e;
}

// n S_bb - S_b^2 of an entry, exactly (see MomEntry)
DEV int32_t mom_db(const MomEntry& m) {
    return m.w > 0.0 ? (int32_t)rint(1.0 / (m.w * m.w)) : 0;
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

// The two windows are loaded once as aligned dwords (NB rows of NW+1 quads,
// the same reads wave_score issues) and re-aligned in registers; the numpy-
// order arithmetic then runs on registers instead of re-reading ~6 bytes of
// the stack per pixel (the guard path used to wait on ~700 dependent loads).
template <int WID>
__device__ __noinline__ double exact_ncc_stack(const SceneDev sc, int R, int v, int q, int r) {
    constexpr int NB = 2 * WID + 1, NW = (NB + 3) / 4;
    const int q0 = q - WID, o = q0 & 3;
    const int64_t vstride = (int64_t)sc.V * 4;
    const uint8_t* p0 = sc.stack + (int64_t)(r - WID) * sc.row_bytes + (int64_t)(q0 >> 2) * vstride;
    uint32_t wa[NB][NW], wb[NB][NW];
#pragma unroll
    for (int row = 0; row < NB; ++row) {
        uint32_t da[NW + 1], db[NW + 1];
#pragma unroll
        for (int j = 0; j <= NW; ++j) {
            da[j] = *(const uint32_t*)(p0 + (int64_t)row * sc.row_bytes + j * vstride + R * 4);
            db[j] = *(const uint32_t*)(p0 + (int64_t)row * sc.row_bytes + j * vstride + v * 4);
        }
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            wa[row][j] = __builtin_amdgcn_alignbyte(da[j + 1], da[j], o);
            wb[row][j] = __builtin_amdgcn_alignbyte(db[j + 1], db[j], o);
        }
    }
    auto A = [&](int i) -> int { return (int)((wa[i / NB][(i % NB) >> 2] >> (8 * ((i % NB) & 3))) & 0xffu); };
    auto B = [&](int i) -> int { return (int)((wb[i / NB][(i % NB) >> 2] >> (8 * ((i % NB) & 3))) & 0xffu); };
    return exact_ncc_fixed<NB * NB>(A, B);
}

// Wave-wide binary64 sum without LDS: DPP butterflies inside each row of 16
// lanes, then the four row sums combined from SGPRs.  Result in every lane.
template <int CTRL>
DEV double dpp_f64(double x) {
    // bound_ctrl: every source lane of these patterns exists, so no "old" value
    // (and no v_mov to materialise it) is needed
    const unsigned long long u = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

// row_bcast:15 / row_bcast:31 (GFX9 DPP): rows in ROWMASK receive the last lane
// of the row before / of row 1; the other rows get 0
template <int CTRL, int ROWMASK>
DEV double dpp_bcast_f64(double x) {
    const unsigned long long u = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROWMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROWMASK, 0xf, false);
    return __longlong_as_double(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

DEV double wave_sum_dpp(double x) {
    x += dpp_f64<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dpp_f64<0x4E>(x);    // quad_perm [2,3,0,1]
    x += dpp_f64<0x141>(x);   // row_half_mirror
    x += dpp_f64<0x140>(x);   // row_mirror: every lane holds its row's sum
    x += dpp_bcast_f64<0x142, 0xa>(x);   // rows 1, 3 += rows 0, 2
    x += dpp_bcast_f64<0x143, 0xc>(x);   // rows 2, 3 += rows 0+1: lane 63 holds the total
    const unsigned long long u = __double_as_longlong(x);
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, 63);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

DEV double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// One window row of every view of this lane: align, broadcast the reference
// view's words, accumulate S_ab (dot4), S_bb (dot4), S_b (sad).
template <int NS, int NW, int ND, uint32_t LASTMASK, class Fetch>
DEV void wave_row(Fetch&& fetch, int row, int o, int V, int Rs, int Rl, int lane, uint32_t* Sb,
                  uint32_t* Sbb, uint32_t* Sab) {
    uint32_t w[NS][NW];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int v = lane + 64 * s;
        uint32_t d[ND];
        if (NS == 1 || v < V) {
#pragma unroll
            for (int j = 0; j < ND; ++j) d[j] = fetch(s, row, j);
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

// One wave scores one candidate whose window sits at (q, r) of every view
// (the reference samples all views at view R's pixel, MVS2.py:68).
// Lane l handles views l, l+64, ... (NS slots).  fetch(s, row, j) returns the
// j-th dword (4 pixels of this lane's view of slot s) of window row `row`,
// counted from the quad holding column q - WID; o = (q - WID) & 3.
// Lane 0 of the wave writes mask/count/avg.
// Variants (A/B-able at run time, see mvs_launch_score_tiled):
//   EPI 2: decision from exact-integer-fed squared comparison (no sqrt/div),
//          relative band 1e-8 -> numpy order; value (for avg) by rsq+Newton
//   EPI 0: decision from the binary64 closed form (guard 1e-9 -> numpy order)
//   EPI 1: decision from a binary32 closed form (|err| < 4e-7; guard 1e-5 ->
//          binary64 -> guard 1e-9 -> numpy order); binary64 only for lanes in
//          the guard and, when avg is wanted, for passing lanes
//   REF 0: reference-view words broadcast with v_readlane
//   REF 1: reference-view words re-read by every lane (same LDS address = broadcast)
template <int WID, int NS, bool UNROLL = false, int EPI = 2, int REF = 0, class Fetch,
          class FetchRef>
DEV void wave_score_core(const SceneDev& sc, int R, int q, int r, double thr, Fetch&& fetch,
                         FetchRef&& fref, uint64_t* mask_out, int32_t* count_out,
                         double* avg_out, int32_t* exact_hits) {
    constexpr int NB = 2 * WID + 1;
    constexpr int NPX = NB * NB;
    constexpr int NW = (NB + 3) / 4;
    constexpr int ND = NW + 1;
    constexpr uint32_t LASTMASK = (NB % 4 == 0) ? 0xffffffffu : ((1u << (8 * (NB % 4))) - 1u);
    const int lane = threadIdx.x & 63;
    const int o = (q - WID) & 3;
    const int V = sc.V;
    const int Rs = R >> 6, Rl = R & 63;

    uint32_t Sb[NS], Sbb[NS], Sab[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) Sb[s] = Sbb[s] = Sab[s] = 0;

    if constexpr (UNROLL) {
        // LDS-resident rows: issue every read of the window first, then run
        // the dot products on NW independent accumulator chains.
        static_assert(NS == 1, "unrolled path is single-slot");
        uint32_t d[NB][ND];
#pragma unroll
        for (int row = 0; row < NB; ++row)
#pragma unroll
            for (int j = 0; j < ND; ++j) d[row][j] = fetch(0, row, j);
        uint32_t ab[NW], bb[NW], b1[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) ab[j] = bb[j] = b1[j] = 0;
#pragma unroll
        for (int row = 0; row < NB; ++row) {
            uint32_t w[NW], a[NW];
#pragma unroll
            for (int j = 0; j < NW; ++j) w[j] = __builtin_amdgcn_alignbyte(d[row][j + 1], d[row][j], o);
            w[NW - 1] &= LASTMASK;
            if constexpr (REF == 0) {
#pragma unroll
                for (int j = 0; j < NW; ++j) a[j] = __builtin_amdgcn_readlane(w[j], Rl);
            } else {
                uint32_t e[ND];
#pragma unroll
                for (int j = 0; j < ND; ++j) e[j] = fref(row, j);
#pragma unroll
                for (int j = 0; j < NW; ++j) a[j] = __builtin_amdgcn_alignbyte(e[j + 1], e[j], o);
                a[NW - 1] &= LASTMASK;
            }
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                ab[j] = __builtin_amdgcn_udot4(a[j], w[j], ab[j], false);
                bb[j] = __builtin_amdgcn_udot4(w[j], w[j], bb[j], false);
                b1[j] = __builtin_amdgcn_sad_u8(w[j], 0u, b1[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            Sab[0] += ab[j];
            Sbb[0] += bb[j];
            Sb[0] += b1[j];
        }
    }
#pragma unroll 1
    for (int row = 0; row < (UNROLL ? 0 : NB); ++row) {
        uint32_t w[NS][NW];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int v = lane + 64 * s;
            uint32_t d[ND];
            if (NS == 1 || v < V) {
#pragma unroll
                for (int j = 0; j < ND; ++j) d[j] = fetch(s, row, j);
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
        const bool live = v < V && v != R && da > 0 && db > 0;   // da/db == 0: ctNcc nan -> reject
        auto ncc64 = [&]() {
            return (double)((int64_t)NPX * num) / ((double)(NPX - 1) * sqrt((double)da * (double)db));
        };
        if constexpr (EPI == 2) {
            // Decision without sqrt/div: for thr >= 0.01, ncc > thr  <=>  L > 0 and
            // L^2 > thr^2 (n-1)^2 da db  with L = n*num (exact in binary64).  The
            // products carry < 1e-15 relative error; a relative band of 1e-8
            // (|ncc - thr| < ~thr*5e-9) goes to the numpy-order path, far wider
            // than the reference's own rounding (< 1e-12).
            if (live) {
                if (thr >= 0.01) {
                    const double L = (double)((int64_t)NPX * num);
                    if (L > 0.0) {
                        const double tk = thr * (double)(NPX - 1);
                        const double rhs = (tk * tk) * ((double)da * (double)db);
                        const double diff = L * L - rhs;
                        if (fabs(diff) <= 1e-8 * rhs) {
                            ncc = exact_ncc_stack<WID>(sc, R, v, q, r);
                            atomicAdd(exact_hits, 1);
                            pass = ncc > thr;
                        } else {
                            pass = diff > 0.0;
                            if (pass && avg_out) {
                                // avg_ncc_score value only: rsq + two Newton steps
                                const double D = (double)da * (double)db;
                                double y = __builtin_amdgcn_rsq(D);
                                y = y * (1.5 - 0.5 * D * y * y);
                                y = y * (1.5 - 0.5 * D * y * y);
                                ncc = L * y * (1.0 / (double)(NPX - 1));
                            }
                        }
                    }
                } else {
                    ncc = ncc64();
                    if (fabs(ncc - thr) <= kGuard) {
                        ncc = exact_ncc_stack<WID>(sc, R, v, q, r);
                        atomicAdd(exact_hits, 1);
                    }
                    pass = ncc > thr;
                }
            }
        } else if constexpr (EPI == 0) {
            if (live) {
                ncc = ncc64();
                if (fabs(ncc - thr) <= kGuard) {
                    ncc = exact_ncc_stack<WID>(sc, R, v, q, r);
                    atomicAdd(exact_hits, 1);
                }
                pass = ncc > thr;
            }
        } else {
            if (live) {
                const float n32 = (float)((int64_t)NPX * num) /
                                  ((float)(NPX - 1) * sqrtf((float)da * (float)db));
                const float thr32 = (float)thr;
                if (fabsf(n32 - thr32) <= 1e-5f) {
                    ncc = ncc64();
                    if (fabs(ncc - thr) <= kGuard) {
                        ncc = exact_ncc_stack<WID>(sc, R, v, q, r);
                        atomicAdd(exact_hits, 1);
                    }
                    pass = ncc > thr;
                } else {
                    pass = n32 > thr32;
                    if (pass && avg_out) ncc = ncc64();
                }
            }
        }
        const uint64_t m = __ballot(pass);
        // NS slots can exceed the candidate's ceil(V/64) mask words (NS = 4 for
        // 128 < V <= 192): only the words that exist are written
        if (lane == 0 && 64 * s < V) mask_out[s] = m;
        cnt += __popcll(m);
        acc += pass ? ncc : 0.0;
    }
    if ((EPI != 0 && !avg_out) || cnt == 0) {
        if (lane == 0) {
            *count_out = cnt;
            if (avg_out) *avg_out = 0.0;
        }
        return;
    }
    const double tot = wave_sum(acc);
    if (lane == 0) {
        *count_out = cnt;
        if (avg_out) *avg_out = cnt > 0 ? tot / cnt : 0.0;
    }
}

// Direct variant: window rows gathered straight from the HBM-resident stack.
template <int WID, int NS>
DEV void wave_score(const SceneDev& sc, int R, int q, int r, double thr, uint64_t* mask_out,
                    int32_t* count_out, double* avg_out, int32_t* exact_hits) {
    const int lane = threadIdx.x & 63;
    const int k0 = (q - WID) >> 2;
    const int64_t vstride = (int64_t)sc.V * 4;
    const uint8_t* p0 = sc.stack + (int64_t)(r - WID) * sc.row_bytes + (int64_t)k0 * vstride;
    auto fetch = [&](int s, int row, int j) -> uint32_t {
        return *(const uint32_t*)(p0 + (int64_t)row * sc.row_bytes + j * vstride + (lane + 64 * s) * 4);
    };
    auto fref = [&](int, int) -> uint32_t { return 0u; };
    wave_score_core<WID, NS>(sc, R, q, r, thr, fetch, fref, mask_out, count_out, avg_out, exact_hits);
}

template <int NS>
DEV void wave_score_empty(uint64_t* mask_out, int32_t* count_out, double* avg_out, int words) {
    const int lane = threadIdx.x & 63;
    if (lane < NS && lane < words) mask_out[lane] = 0;
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
        wave_score_empty<NS>(a.mask + cand * words, a.count + cand, a.avg ? a.avg + cand : nullptr, words);
        return;
    }
    q = __builtin_amdgcn_readfirstlane(q);
    r = __builtin_amdgcn_readfirstlane(r);
    wave_score<WID, NS>(sc, R, q, r, a.thr, a.mask + cand * words, a.count + cand,
                        a.avg ? a.avg + cand : nullptr, a.exact_hits);
}

// ---------------------------------------------------------------------------
// Tiled scorer: candidates binned by the TWxTH pixel tile of their window
// centre; a workgroup stages the tile's window region of ALL views in LDS
// (a straight copy of the stack's [row][quad][view] layout) and its waves
// score the tile's candidates from LDS.
// ---------------------------------------------------------------------------
constexpr int kTW = 16, kTH = 8, kChunk = 512, kTiledBlocks = 2048;

template <int WID>
struct TileGeom {
    static constexpr int NB = 2 * WID + 1;
    static constexpr int NW = (NB + 3) / 4;
    static constexpr int KQ0 = -((WID + 3) / 4);                 // first quad, relative to x0/4
    static constexpr int KQL = ((kTW - 1 - WID) >> 2) + NW;        // last quad read, relative
    static constexpr int NQ = KQL - KQ0 + 1;
    static constexpr int ROWS = kTH + 2 * WID;
};

// k_bin: project every candidate (FP64, reference order), test its window,
// and rank it inside its tile.  Ranks come from an LDS histogram per block
// (one global atomic per non-empty (block, tile) pair), not from a global
// atomic per candidate.
constexpr int kBinBlock = 1024, kBinPerDefault = 4;

template <int kBinPer>
__global__ __launch_bounds__(kBinBlock) void k_bin(const SceneDev sc, const ScoreArgs a,
                                                   const TiledArgs t, int wid) {
    extern __shared__ int32_t hist[];      // [ntiles] local counts, then global bases
    const int words = (sc.V + 63) >> 6;
    for (int b = threadIdx.x; b < t.ntiles; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kBinBlock * kBinPer;
    int tl[kBinPer], lr[kBinPer];
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
        const int64_t i = base + (int64_t)k * kBinBlock + threadIdx.x;
        tl[k] = -1;
        if (i >= a.n) continue;
        const int R = a.ref[i];
        const double c[3] = {a.c[3 * i], a.c[3 * i + 1], a.c[3 * i + 2]};
        double px, py;
        project(sc.cams[R], c, px, py);
        a.xy[2 * i] = px;
        a.xy[2 * i + 1] = py;
        int q, r;
        if (!window_ok(sc, px, py, wid, &q, &r)) {
            for (int w = 0; w < words; ++w) a.mask[i * words + w] = 0;
            a.count[i] = 0;
            if (a.avg) a.avg[i] = 0.0;
            t.cand_key[i] = -1;
            continue;
        }
        const int tile = (r / t.th) * t.ntx + (q / t.tw);
        tl[k] = tile;
        t.cand_pk[i] = q | (r << 11) | (R << 22);
        lr[k] = atomicAdd(&hist[tile], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < t.ntiles; b += blockDim.x) {
        const int c = hist[b];
        hist[b] = c ? atomicAdd(&t.tile_count[b], c) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
        const int64_t i = base + (int64_t)k * kBinBlock + threadIdx.x;
        if (tl[k] < 0) continue;
        t.cand_key[i] = tl[k];
        t.cand_rank[i] = hist[tl[k]] + lr[k];
    }
}

// candidates per k_bin thread (MVS_BIN_PER = 1/2/4/8, read once; A/B only):
// fewer per thread = more blocks, but one more global atomic per (block, tile)
static int bin_per() {
    static const int p = [] {
        const char* e = getenv("MVS_BIN_PER");
        const int v = e ? atoi(e) : kBinPerDefault;
        return (v == 1 || v == 2 || v == 4 || v == 8) ? v : kBinPerDefault;
    }();
    return p;
}

static void launch_bin(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, int wid, hipStream_t s) {
    const int per = bin_per();
    const int64_t per_block = (int64_t)kBinBlock * per;
    const int nbin = (int)((a->n + per_block - 1) / per_block);
    const size_t lds = (size_t)t->ntiles * 4;
    switch (per) {
        case 1: hipLaunchKernelGGL(k_bin<1>, dim3(nbin), dim3(kBinBlock), lds, s, *sc, *a, *t, wid); break;
        case 2: hipLaunchKernelGGL(k_bin<2>, dim3(nbin), dim3(kBinBlock), lds, s, *sc, *a, *t, wid); break;
        case 8: hipLaunchKernelGGL(k_bin<8>, dim3(nbin), dim3(kBinBlock), lds, s, *sc, *a, *t, wid); break;
        default: hipLaunchKernelGGL(k_bin<4>, dim3(nbin), dim3(kBinBlock), lds, s, *sc, *a, *t, wid); break;
    }
}

// Exclusive scans of tile counts and work items (one workgroup), and the
// work-item list in longest-first order: all full chunks (tile-major), then
// the partial chunks by decreasing candidate count.  A dynamic queue handed
// out in that order ends on its shortest items, which trims the tail where
// a few workgroups still run while the rest of the chip idles.
// Inclusive scan of N values per thread over a 1024-thread block: wave scans
// by __shfl_up, the 16 wave totals scanned by one wave, two barriers.
template <int N>
DEV void block_scan_1024(int32_t (&v)[N], int32_t* wtot /* LDS, 16 * N */) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t y = __shfl_up(v[k], off, 64);
            if (lane >= off) v[k] += y;
        }
    if (lane == 63)
#pragma unroll
        for (int k = 0; k < N; ++k) wtot[wave * N + k] = v[k];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            int32_t x = lane < 16 ? wtot[lane * N + k] : 0;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                const int32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            if (lane < 16) wtot[lane * N + k] = x;
        }
    }
    __syncthreads();
    if (wave > 0)
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] += wtot[(wave - 1) * N + k];
}

// Exclusive scans of tile counts and work items (one workgroup), and the
// work-item list in longest-first order: all full chunks (tile-major), then
// the partial chunks by decreasing candidate count.  A dynamic queue handed
// out in that order ends on its shortest items, which trims the tail where
// a few workgroups still run while the rest of the chip idles.
__global__ __launch_bounds__(1024) void k_tile_scan(const TiledArgs t) {
    __shared__ int32_t wtot[16 * 3];
    __shared__ int32_t tot[3];
    __shared__ int32_t hist[1025];                 // partial-chunk sizes (chunk <= 1024)
    const int tid = threadIdx.x;
    const int per = (t.ntiles + 1023) / 1024;
    const int b = tid * per, e = min(b + per, t.ntiles);
    int32_t v3[3] = {0, 0, 0};                     // candidates, items, full chunks of my tiles
    for (int k = b; k < e; ++k) {
        const int c = t.tile_count[k];
        v3[0] += c;
        v3[1] += (c + t.chunk - 1) / t.chunk;
        v3[2] += c / t.chunk;
    }
    const int32_t own[3] = {v3[0], v3[1], v3[2]};
    for (int s = tid; s <= 1024; s += 1024) hist[s] = 0;
    block_scan_1024<3>(v3, wtot);
    if (tid == 1023) { tot[0] = v3[0]; tot[1] = v3[1]; tot[2] = v3[2]; }
    if (t.items)
        for (int k = b; k < e; ++k) {
            const int rem = t.tile_count[k] % t.chunk;
            if (rem) atomicAdd(&hist[rem], 1);
        }
    __syncthreads();
    const int32_t n_full = tot[2];
    {
        // descending exclusive prefix, hist[s] = partials longer than s, as a
        // scan over the sizes in reverse order (thread i <-> size chunk-1-i)
        const int nsz = t.chunk - 1;
        const int32_t mine = (t.items && tid < nsz) ? hist[t.chunk - 1 - tid] : 0;
        int32_t r1[1] = {mine};
        __syncthreads();                            // everyone has read hist before it is rewritten
        block_scan_1024<1>(r1, wtot);
        if (t.items && tid < nsz) hist[t.chunk - 1 - tid] = r1[0] - mine;
        __syncthreads();
    }
    int32_t rc = v3[0] - own[0], ri = v3[1] - own[1], rf = v3[2] - own[2];
    for (int k = b; k < e; ++k) {
        t.tile_off[k] = rc;
        t.item_off[k] = ri;
        const int c = t.tile_count[k];
        rc += c;
        ri += (c + t.chunk - 1) / t.chunk;
        if (t.items) {
            const int full = c / t.chunk, rem = c - full * t.chunk;
            for (int j = 0; j < full; ++j) t.items[rf + j] = make_int2(k, j);
            rf += full;
            if (rem) t.items[n_full + atomicAdd(&hist[rem], 1)] = make_int2(k, full);
        }
        t.tile_count[k] = 0;          // clean for the next batch's k_bin
    }
    if (tid == 1023) {
        t.tile_off[t.ntiles] = tot[0];
        t.item_off[t.ntiles] = tot[1];
    }
    // work-queue heads and the fix-list length start this batch at zero
    if (tid == 0) {
        t.tile_count[t.ntiles] = 0;
        t.tile_count[t.ntiles + 1] = 0;
    }
    if (t.xq && tid < 8) t.xq[tid] = 0;
}

__global__ void k_scatter(const ScoreArgs a, const TiledArgs t) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int tile = t.cand_key[i];
        if (tile >= 0) t.sorted[t.tile_off[tile] + t.cand_rank[i]] = make_int2((int32_t)i, t.cand_pk[i]);
    }
}

// LDS image of a tile region: [row][quad][64 view slots] dwords, so every
// window dword of lane v sits at a compile-time offset from one base address
// (ds_read2st64_b32 pairs), and the 64 lanes of a read hit 64 banks.
template <int WID, int EPI, int REF>
__global__ __launch_bounds__(256) void k_score_tiled(const SceneDev sc, const ScoreArgs a,
                                                     const TiledArgs t) {
    using G = TileGeom<WID>;
    constexpr int QS = 64;                 // dwords per (row, quad)
    constexpr int RS = G::NQ * QS;         // dwords per region row
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int V = sc.V;                    // <= 64
    const int n_items = t.item_off[t.ntiles];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
        int lo = 0, hi = t.ntiles;         // tile = last k with item_off[k] <= item
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (t.item_off[mid] <= item) lo = mid; else hi = mid;
        }
        const int tile = lo;
        const int chunk = item - t.item_off[tile];
        const int cb = t.tile_off[tile] + chunk * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int y0 = ty * kTH - WID;                 // first region row
        const int kq0 = tx * (kTW / 4) + G::KQ0;       // first region quad
        // stage the region: 16-B chunks (4 views of one (row, quad)); each thread
        // issues all its loads before its LDS writes so the fetches overlap
        if ((V & 3) == 0) {
            const int cpq = V >> 2, cpr = G::NQ * cpq, total = G::ROWS * cpr;
            for (int base = 0; base < total; base += 8 * 256) {
                uint4 buf[8];
                int dst[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int k = base + u * 256 + (int)threadIdx.x;
                    dst[u] = -1;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (k < total) {
                        const int ry = k / cpr, rem = k - ry * cpr;
                        const int kq = rem / cpq, vq = rem - kq * cpq;
                        const int y = y0 + ry, gq = kq0 + kq;
                        if (y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                            buf[u] = *(const uint4*)(sc.stack + (int64_t)y * sc.row_bytes +
                                                      (int64_t)gq * V * 4 + vq * 16);
                        dst[u] = (ry * G::NQ + kq) * QS + vq * 4;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (dst[u] >= 0) *(uint4*)(lds + dst[u]) = buf[u];
            }
        } else {
            for (int pq = wave; pq < G::ROWS * G::NQ; pq += 4) {
                const int ry = pq / G::NQ, kq = pq - ry * G::NQ;
                const int y = y0 + ry, gq = kq0 + kq;
                uint32_t val = 0;
                if (lane < V && y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                    val = *(const uint32_t*)(sc.stack + (int64_t)y * sc.row_bytes + (int64_t)gq * V * 4 + lane * 4);
                lds[pq * QS + lane] = val;
            }
        }
        __syncthreads();
        int2 nxt = cb + wave < ce ? t.sorted[cb + wave] : make_int2(0, 0);
        for (int j = cb + wave; j < ce; j += 4) {
            const int2 cur = nxt;
            if (j + 4 < ce) nxt = t.sorted[j + 4];
            const int i = __builtin_amdgcn_readfirstlane(cur.x);
            const int pk = __builtin_amdgcn_readfirstlane(cur.y);
            const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
            const int ry0 = r - WID - y0;
            const int k0 = ((q - WID) >> 2) - kq0;
            const uint32_t* basep = lds + ry0 * RS + k0 * QS + lane;
            auto fetch = [&](int, int row, int jj) -> uint32_t { return basep[row * RS + jj * QS]; };
            const uint32_t* refp = basep - lane + R;
            auto fref = [&](int row, int jj) -> uint32_t { return refp[row * RS + jj * QS]; };
            wave_score_core<WID, 1, true, EPI, REF>(sc, R, q, r, a.thr, fetch, fref, a.mask + i,
                                                    a.count + i, a.avg ? a.avg + i : nullptr,
                                                    a.exact_hits);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Scene-level precompute: view-major gray copy and per-view window moments
// ---------------------------------------------------------------------------
__global__ void k_build_gv(const uint8_t* __restrict__ stack, uint8_t* __restrict__ gv, int V, int H,
                           int W, int Wq, int Wp) {
    const int64_t total = (int64_t)V * H * Wp;
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(id % Wp);
        const int64_t vy = id / Wp;
        const int y = (int)(vy % H), v = (int)(vy / H);
        uint8_t g = 0;
        if (x < W) g = stack[(int64_t)y * Wq * V * 4 + (int64_t)(x >> 2) * V * 4 + v * 4 + (x & 3)];
        gv[id] = g;
    }
}

// (S_b, S_bb, 1/sqrt(n S_bb - S_b^2)) of every view's window at every valid
// centre; one thread per (pixel, view), rows summed from the aligned words of
// the stack.
template <int WID>
__global__ void k_moments(const SceneDev sc, MomEntry* __restrict__ mom) {
    constexpr int NB = 2 * WID + 1, NW = (NB + 3) / 4;
    constexpr uint32_t LASTMASK = (NB % 4 == 0) ? 0xffffffffu : ((1u << (8 * (NB % 4))) - 1u);
    const int64_t total = (int64_t)sc.H * sc.W * sc.V;
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int v = (int)(id % sc.V);
        const int64_t p = id / sc.V;
        const int x = (int)(p % sc.W), y = (int)(p / sc.W);
        MomEntry out{0.0, 0u};
        if (y - WID >= 0 && y + WID + 1 < sc.H && x - WID > 0 && x + WID + 1 < sc.W) {
            const int q0 = x - WID, k0 = q0 >> 2, o = q0 & 3;
            uint32_t sb = 0, sbb = 0;
            for (int row = 0; row < NB; ++row) {
                const uint8_t* pr = sc.stack + (int64_t)(y - WID + row) * sc.row_bytes +
                                    (int64_t)k0 * sc.V * 4 + v * 4;
                uint32_t d[NW + 1];
#pragma unroll
                for (int j = 0; j <= NW; ++j) d[j] = *(const uint32_t*)(pr + (int64_t)j * sc.V * 4);
#pragma unroll
                for (int j = 0; j < NW; ++j) {
                    uint32_t w = __builtin_amdgcn_alignbyte(d[j + 1], d[j], o);
                    if (j == NW - 1) w &= LASTMASK;
                    sb = __builtin_amdgcn_sad_u8(w, 0u, sb);
                    sbb = __builtin_amdgcn_udot4(w, w, sbb, false);
                }
            }
            const int64_t db = (int64_t)(NB * NB) * sbb - (int64_t)sb * sb;
            out.sb = sb;
            out.w = db > 0 ? 1.0 / sqrt((double)db) : 0.0;
        }
        uint32_t* o = (uint32_t*)mom + 3 * id;
        const unsigned long long wb = __double_as_longlong(out.w);
        o[0] = (uint32_t)wb;
        o[1] = (uint32_t)(wb >> 32);
        o[2] = out.sb;
    }
}

// Tiled scorer, v3: S_b/S_bb from the scene moments; S_ab from the
// unaligned window quads in LDS against the reference view's quads loaded
// by SMEM from the view-major copy and masked to the window (SALU) -- the
// only per-row VALU work is NQW v_dot4_u32_u8.
using cgu32 = __attribute__((address_space(4))) const uint32_t;

// S_ab over the (2WID+1)^2 window whose first column sits at byte O of the
// first quad: raw quads of this lane's view (own) against the reference
// view's quads (ref, LDS broadcast) masked to the window at compile time --
// interior quads need no mask, quads outside the window are skipped.
template <int WID, int O>
struct QuadMasks {
    static constexpr int NB = 2 * WID + 1;
    static constexpr int NQ = (O + NB + 3) / 4;
    static constexpr uint32_t mask(int jj) {
        const int st0 = O - 4 * jj, en0 = O + NB - 4 * jj;
        const int st = st0 < 0 ? 0 : (st0 > 4 ? 4 : st0);
        const int en = en0 < 0 ? 0 : (en0 > 4 ? 4 : en0);
        const uint32_t hiM = en >= 4 ? 0xffffffffu : ((1u << (8 * en)) - 1u);
        const uint32_t loM = (1u << (8 * st)) - 1u;
        return en > st ? (hiM & ~loM) : 0u;
    }
};

using lds_u32 = __attribute__((address_space(3))) const uint32_t;

// The reference quads sit at the same strides (RRS, RQS) = (RS, QS) when they
// come from the region image, or in a per-wave [row][4] slot (RRS 4, RQS 1).
template <int WID, int O, int RS, int QS, int RRS = RS, int RQS = QS>
DEV uint32_t sab_rows(const uint32_t* own_g, const uint32_t* ref_g) {
    using M = QuadMasks<WID, O>;
    constexpr int NB = 2 * WID + 1;
    uint32_t d[NB][M::NQ], e[NB][M::NQ];
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) {
        // one base register per quad column: the rows are RS dwords apart (a
        // multiple of 64 when RS = 8*48), so each column's 11 rows pair up
        // into ds_read2st64_b32 off that base with no further address math
        lds_u32* o = (lds_u32*)own_g + jj * QS;
        lds_u32* r = (lds_u32*)ref_g + jj * RQS;
        asm volatile("" : "+v"(o));
        asm volatile("" : "+v"(r));
#pragma unroll
        for (int row = 0; row < NB; ++row) {
            d[row][jj] = o[row * RS];
            e[row][jj] = r[row * RRS];
        }
    }
    uint32_t ab[M::NQ];
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) ab[jj] = 0;
#pragma unroll
    for (int row = 0; row < NB; ++row)
#pragma unroll
        for (int jj = 0; jj < M::NQ; ++jj) {
            const uint32_t m = M::mask(jj);
            const uint32_t am = (m == 0xffffffffu) ? e[row][jj] : (e[row][jj] & m);
            ab[jj] = __builtin_amdgcn_udot4(am, d[row][jj], ab[jj], false);
        }
    uint32_t sum = 0;
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) sum += ab[jj];
    return sum;
}

// Row-streamed S_ab for k_score_tiled5: window rows in groups of RG, the
// next group's reads issued before the current group's dot products, an
// empty asm tying their addresses to the accumulators keeping the compiler
// from hoisting every read to the front -- 16-32 live window VGPRs instead of
// 88, so more waves per SIMD fit.
template <int WID, int O, int RS, int QS>
DEV uint32_t sab_rows_stream(const uint32_t* own_g, const uint32_t* ref_g) {
    using M = QuadMasks<WID, O>;
    constexpr int NB = 2 * WID + 1;
    // rows per group: pairs (ds_read2st64) while the double buffer stays
    // small, single rows (ds_read_b32, the same LDS cycles per dword) at wid 5
    constexpr int RG = M::NQ >= 4 ? 1 : 2;
    constexpr int NG = (NB + RG - 1) / RG;
    uint32_t d[2][RG][M::NQ], e[2][RG][M::NQ];
    lds_u32* ob = (lds_u32*)own_g;
    lds_u32* rb = (lds_u32*)ref_g;
    auto load = [&](int g, uint32_t (&dd)[RG][M::NQ], uint32_t (&ee)[RG][M::NQ]) {
#pragma unroll
        for (int h = 0; h < RG; ++h) {
            const int row = RG * g + h;
#pragma unroll
            for (int jj = 0; jj < M::NQ; ++jj) {
                dd[h][jj] = row < NB ? ob[row * RS + jj * QS] : 0u;
                ee[h][jj] = row < NB ? rb[row * RS + jj * QS] : 0u;
            }
        }
    };
    uint32_t ab[M::NQ];
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) ab[jj] = 0;
    load(0, d[0], e[0]);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) {
            // the next group's addresses "depend" on the accumulators as they
            // stand after group g-1: its reads cannot be hoisted further up, so
            // at most two groups of window words are live; pinning every
            // accumulator (not only ab[0]) also stops the scheduler from
            // sinking the group-g ALU work below the next loads (12 VGPR
            // spills at wid 5 without it, none with it)
#pragma unroll
            for (int jj = 0; jj < M::NQ; ++jj) asm volatile("" : "+v"(ab[jj]));
            asm volatile("" : "+v"(ob), "+v"(rb) : "v"(ab[0]));
            load(g + 1, d[(g + 1) & 1], e[(g + 1) & 1]);
        }
#pragma unroll
        for (int h = 0; h < RG; ++h) {
            if (RG * g + h < NB) {
#pragma unroll
                for (int jj = 0; jj < M::NQ; ++jj) {
                    const uint32_t m = M::mask(jj);
                    const uint32_t ev = e[g & 1][h][jj];
                    const uint32_t am = (m == 0xffffffffu) ? ev : (ev & m);
                    ab[jj] = __builtin_amdgcn_udot4(am, d[g & 1][h][jj], ab[jj], false);
                }
            }
        }
    }
    uint32_t sum = 0;
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) sum += ab[jj];
    return sum;
}

// Same with the reference view's window quads loaded by SMEM (uniform
// address, s_load) from the view-major copy: no LDS traffic and no VGPRs for
// the reference side; masks applied on the SALU.
template <int WID, int O, int RS, int QS>
DEV uint32_t sab_rows_smem(const uint32_t* own, cgu32* ref, int ref_pitch_dw) {
    using M = QuadMasks<WID, O>;
    constexpr int NB = 2 * WID + 1;
    uint32_t d[NB][M::NQ];
#pragma unroll
    for (int row = 0; row < NB; ++row)
#pragma unroll
        for (int jj = 0; jj < M::NQ; ++jj) d[row][jj] = own[row * RS + jj * QS];
    uint32_t ab[M::NQ];
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) ab[jj] = 0;
#pragma unroll
    for (int row = 0; row < NB; ++row)
#pragma unroll
        for (int jj = 0; jj < M::NQ; ++jj) {
            const uint32_t m = M::mask(jj);
            const uint32_t e = ref[row * ref_pitch_dw + jj];
            const uint32_t am = (m == 0xffffffffu) ? e : (e & m);
            ab[jj] = __builtin_amdgcn_udot4(am, d[row][jj], ab[jj], false);
        }
    uint32_t sum = 0;
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) sum += ab[jj];
    return sum;
}

constexpr int kT3Threads = 256, kT3Waves = kT3Threads / 64;

// 1/k for k = 0..64 (entry 0 unused), correctly rounded at compile time:
// avg_ncc_score = sum * (1/cnt) -- one multiply instead of a binary64 divide.
struct RecipTable {
    double r[65];
    constexpr RecipTable() : r() {
        for (int k = 1; k <= 64; ++k) r[k] = 1.0 / (double)k;
    }
};
__constant__ constexpr RecipTable c_recip{};

// Diagnostic build only (-DMVS_STAMPS): per-workgroup phase times of the
// tiled kernel -- stage, candidates, write-out -- into a side buffer that no
// output depends on.
#ifdef MVS_STAMPS
__device__ unsigned long long g_stamps[4096 * 8];
#define STAMP(k)                                                                          \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        const unsigned long long ts_ = __builtin_amdgcn_s_memtime();                      \
        __builtin_amdgcn_sched_barrier(0);                                                \
        if (threadIdx.x == 0 && blockIdx.x < 4096) {                                      \
            if ((k) == 0) st_prev = ts_;                                                  \
            else { g_stamps[blockIdx.x * 8 + (k)] += ts_ - st_prev; st_prev = ts_; }      \
            if ((k) == 3) g_stamps[blockIdx.x * 8] += 1;                                  \
        }                                                                                 \
    } while (0)
// phase split inside the workgroup's loop (thread 0 = wave 0 only)
#define STAMP_T(var) \
    __builtin_amdgcn_sched_barrier(0); const unsigned long long var = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0)
#define STAMP_ADD(k, t0, t1) \
    do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_stamps[blockIdx.x * 8 + (k)] += (t1) - (t0); } while (0)
#else
#define STAMP(k) do { } while (0)
#define STAMP_T(var) do { } while (0)
#define STAMP_ADD(k, t0, t1) do { } while (0)
#endif

template <int WID, int QS, int REFSRC>
__global__ __launch_bounds__(kT3Threads, 4) void k_score_tiled3(const SceneDev sc, const ScoreArgs a,
                                                                const TiledArgs t) {
    using G = TileGeom<WID>;
    constexpr int NB = 2 * WID + 1;
    constexpr int NPX = NB * NB;
    // QS: dwords per (row, quad) slot of the LDS image (= V when V == 48)
    constexpr int RS = G::NQ * QS;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int V = sc.V;
    const int n_items = t.item_off[t.ntiles];
    // wave index as an SGPR: the candidate loop, its SMEM loads and the
    // alignment switch below are then scalar control flow
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const MomEntry* __restrict__ mom = sc.mom[WID];
    // output staging behind the region image (chunk <= kChunk candidates)
    uint64_t* o_mask = (uint64_t*)(lds + G::ROWS * RS);
    double* o_avg = (double*)(o_mask + t.chunk);
    int32_t* o_cnt = (int32_t*)(o_avg + t.chunk);
    int32_t* o_idx = o_cnt + t.chunk;
    __shared__ int s_item;
#ifdef MVS_STAMPS
    unsigned long long st_prev = 0;
#endif
    for (;;) {
        // dynamic work queue: the next (tile, chunk) item for this workgroup
        if (threadIdx.x == 0) s_item = atomicAdd(&t.tile_count[t.ntiles], 1);
        __syncthreads();
        // uniform from here on: tile bounds and offsets live in SGPRs
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= n_items) break;
        STAMP(0);
        // longest-first item list (k_tile_scan); uniform address -> scalar load
        const unsigned long long itv =
            *(const __attribute__((address_space(4))) unsigned long long*)(t.items + item);
        const int tile = (int)(uint32_t)itv, chunk = (int)(uint32_t)(itv >> 32);
        const int cb = t.tile_off[tile] + chunk * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int y0 = ty * kTH - WID;
        const int kq0 = tx * (kTW / 4) + G::KQ0;
        {
            const int cpq = V >> 2, cpr = G::NQ * cpq, total = G::ROWS * cpr;
            for (int base = 0; base < total; base += 8 * kT3Threads) {
                uint4 buf[8];
                int dst[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int k = base + u * kT3Threads + (int)threadIdx.x;
                    dst[u] = -1;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (k < total) {
                        const int ry = k / cpr, rem = k - ry * cpr;
                        const int kq = rem / cpq, vq = rem - kq * cpq;
                        const int y = y0 + ry, gq = kq0 + kq;
                        if (y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                            buf[u] = *(const uint4*)(sc.stack + (int64_t)y * sc.row_bytes +
                                                      (int64_t)gq * V * 4 + vq * 16);
                        dst[u] = (ry * G::NQ + kq) * QS + vq * 4;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (dst[u] >= 0) *(uint4*)(lds + dst[u]) = buf[u];
            }
        }
        __syncthreads();
        STAMP(1);
        // Candidates: outputs go to an LDS staging slot and leave the CU after
        // the loop, so no wave ever waits on its own stores (vmcnt counts
        // stores and loads together, in order).  The next candidate's entry
        // (SMEM) and moments (VMEM) are fetched one iteration ahead.
        auto sload = [](const int2* p) -> int2 {   // uniform address -> s_load_dwordx2
            const unsigned long long v = *(const __attribute__((address_space(4))) unsigned long long*)p;
            return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
        };
        int2 cur = cb + wave < ce ? sload(t.sorted + cb + wave) : make_int2(0, 0);
        MomEntry mb_cur{0.0, 0u};
        if (cb + wave < ce) {
            const int pk = cur.y, q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
            if (lane < V) mb_cur = load_mom(mom, (r * sc.W + q) * V + lane);
        }
        for (int j = cb + wave; j < ce; j += kT3Waves) {
            const int2 nxt = j + kT3Waves < ce ? sload(t.sorted + j + kT3Waves) : make_int2(0, 0);
            MomEntry mb_nxt{0.0, 0u};
            if (j + kT3Waves < ce) {
                const int pk = nxt.y, q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
                if (lane < V) mb_nxt = load_mom(mom, (r * sc.W + q) * V + lane);
            }
            const int pk = cur.y;
            const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
            const int q0 = q - WID, o = q0 & 3;
            const int k0 = (q0 >> 2) - kq0;
            const MomEntry mb = mb_cur;
            // the reference view's moments: lane R's entry
            const uint32_t ma_sb = __builtin_amdgcn_readlane(mb.sb, R);
            const uint2 wa2 = make_uint2(__builtin_amdgcn_readlane((uint32_t)__double_as_longlong(mb.w), R),
                                         __builtin_amdgcn_readlane((uint32_t)((uint64_t)__double_as_longlong(mb.w) >> 32), R));
            const double wa = __longlong_as_double(((uint64_t)wa2.y << 32) | wa2.x);
            const uint32_t* basep = lds + (r - WID - y0) * RS + k0 * QS + lane;
            // the reference view's quads: same LDS address in every lane (broadcast)
            const uint32_t* refl = basep - lane + R;
            uint32_t Sab = 0;
            if constexpr (REFSRC == 0) {
                // lanes past the last view issue no LDS reads: at V = 48 that is a
                // quarter of the LDS traffic, and LDS bandwidth is a bound here
                if (lane < V) {
                    switch (o) {   // wave-uniform: window byte offset inside the first quad
                        case 0: Sab = sab_rows<WID, 0, RS, QS>(basep, refl); break;
                        case 1: Sab = sab_rows<WID, 1, RS, QS>(basep, refl); break;
                        case 2: Sab = sab_rows<WID, 2, RS, QS>(basep, refl); break;
                        default: Sab = sab_rows<WID, 3, RS, QS>(basep, refl); break;
                    }
                }
            } else {
                cgu32* refg = (cgu32*)(sc.gv + ((int64_t)R * sc.H + (r - WID)) * sc.Wp + 4 * (q0 >> 2));
                const int pitch = sc.Wp >> 2;
                switch (o) {
                    case 0: Sab = sab_rows_smem<WID, 0, RS, QS>(basep, refg, pitch); break;
                    case 1: Sab = sab_rows_smem<WID, 1, RS, QS>(basep, refg, pitch); break;
                    case 2: Sab = sab_rows_smem<WID, 2, RS, QS>(basep, refg, pitch); break;
                    default: Sab = sab_rows_smem<WID, 3, RS, QS>(basep, refg, pitch); break;
                }
            }
            // num = n S_ab - S_a S_b (|num| < 2^31 for windows up to 11x11: 24-bit
            // multiplies, exact).  With w = 1/sqrt(n S_bb - S_b^2) per (pixel, view)
            // from the moments table, ctNcc * (n-1) = n num w_a w_b; it is
            // compared with thr (n-1).  The three roundings leave < 2e-15 relative
            // error, so a relative band of 1e-8 around the threshold (far wider
            // than the reference's own rounding) goes to k_score_fix, which
            // decides those lanes with the numpy-order ctNcc.
            static_assert(NPX <= 121, "24-bit moment products need NB <= 11");
            const int32_t num = (int32_t)(__umul24(NPX, Sab) - __umul24(ma_sb, mb.sb));
            const bool live = lane < V && lane != R && mb.w > 0.0 && wa > 0.0;
            bool pass = false, guard = false;
            double ncc = 0.0;
            if (live) {
                if (a.thr >= 0.01) {
                    const double tk = a.thr * (double)(NPX - 1);
                    const double z = ((double)num * ((double)NPX * wa)) * mb.w;   // ncc (n-1)
                    guard = fabs(z - tk) <= 1e-8 * tk;
                    pass = z > tk;
                    ncc = z;
                } else {
                    // the reference view's n S_aa - S_a^2 from its (wave-uniform) w: lane R
                    // itself is not live, so its lane value cannot be read back here
                    const int32_t db = mom_db(mb);
                    const int32_t da = mom_db(MomEntry{wa, 0u});
                    ncc = ((double)num * (double)NPX) /
                          ((double)(NPX - 1) * sqrt((double)da * (double)db));
                    guard = fabs(ncc - a.thr) <= kGuard;
                    pass = ncc > a.thr;
                    ncc *= (double)(NPX - 1);
                }
            }
            if (__ballot(guard) != 0 && lane == 0) t.fix_list[atomicAdd(t.fix_count, 1)] = cur.x;
            const uint64_t m = __ballot(pass);
            const int cnt = __popcll(m);
            double avgv = 0.0;
            if (a.avg && cnt)
                avgv = wave_sum_dpp(pass ? ncc : 0.0) * (c_recip.r[cnt] * (1.0 / (double)(NPX - 1)));
            const int slot = j - cb;
            if (lane == 0) {
                o_mask[slot] = m;
                o_avg[slot] = avgv;
                o_cnt[slot] = cnt;
                o_idx[slot] = cur.x;
            }
            cur = nxt;
            mb_cur = mb_nxt;
        }
        __syncthreads();
        STAMP(2);
        for (int k = threadIdx.x; k < ce - cb; k += blockDim.x) {
            const int i = o_idx[k];
            a.mask[i] = o_mask[k];
            a.count[i] = o_cnt[k];
            if (a.avg) a.avg[i] = o_avg[k];
        }
        __syncthreads();
        STAMP(3);
    }
}


// ---------------------------------------------------------------------------
// Tiled scorer v5 (default for wid <= 3; variants 14/15): k_score_tiled3 with 8-wave
// workgroups and row-streamed window reads (sab_rows_stream), so that VGPRs
// (and, at 34 KB of LDS per workgroup, 4 workgroups per CU) allow OCC waves
// per SIMD instead of 4.
constexpr int kT5Threads = 512, kT5Waves = kT5Threads / 64;

template <int WID, int QS, int OCC>
__global__ __launch_bounds__(kT5Threads, OCC) void k_score_tiled5(const SceneDev sc, const ScoreArgs a,
                                                                const TiledArgs t) {
    using G = TileGeom<WID>;
    constexpr int NB = 2 * WID + 1;
    constexpr int NPX = NB * NB;
    // QS: dwords per (row, quad) slot of the LDS image (= V when V == 48)
    constexpr int RS = G::NQ * QS;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int V = sc.V;
    const int n_items = t.item_off[t.ntiles];
    // wave index as an SGPR: the candidate loop, its SMEM loads and the
    // alignment switch below are then scalar control flow
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const MomEntry* __restrict__ mom = sc.mom[WID];
    // output staging behind the region image (chunk <= kChunk candidates)
    uint64_t* o_mask = (uint64_t*)(lds + G::ROWS * RS);
    double* o_avg = (double*)(o_mask + t.chunk);
    int32_t* o_cnt = (int32_t*)(o_avg + t.chunk);
    int32_t* o_idx = o_cnt + t.chunk;
    __shared__ int s_item;
#ifdef MVS_STAMPS
    unsigned long long st_prev = 0;
#endif
    for (;;) {
        // dynamic work queue: the next (tile, chunk) item for this workgroup
        if (threadIdx.x == 0) s_item = atomicAdd(&t.tile_count[t.ntiles], 1);
        __syncthreads();
        // uniform from here on: tile bounds and offsets live in SGPRs
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= n_items) break;
        STAMP(0);
        // longest-first item list (k_tile_scan); uniform address -> scalar load
        const unsigned long long itv =
            *(const __attribute__((address_space(4))) unsigned long long*)(t.items + item);
        const int tile = (int)(uint32_t)itv, chunk = (int)(uint32_t)(itv >> 32);
        const int cb = t.tile_off[tile] + chunk * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int y0 = ty * kTH - WID;
        const int kq0 = tx * (kTW / 4) + G::KQ0;
        {
            const int cpq = V >> 2, cpr = G::NQ * cpq, total = G::ROWS * cpr;
            for (int base = 0; base < total; base += 2 * kT5Threads) {
                uint4 buf[2];
                int dst[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int k = base + u * kT5Threads + (int)threadIdx.x;
                    dst[u] = -1;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (k < total) {
                        const int ry = k / cpr, rem = k - ry * cpr;
                        const int kq = rem / cpq, vq = rem - kq * cpq;
                        const int y = y0 + ry, gq = kq0 + kq;
                        if (y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                            buf[u] = *(const uint4*)(sc.stack + (int64_t)y * sc.row_bytes +
                                                      (int64_t)gq * V * 4 + vq * 16);
                        dst[u] = (ry * G::NQ + kq) * QS + vq * 4;
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    if (dst[u] >= 0) *(uint4*)(lds + dst[u]) = buf[u];
            }
        }
        __syncthreads();
        STAMP(1);
        // Candidates: outputs go to an LDS staging slot and leave the CU after
        // the loop, so no wave ever waits on its own stores (vmcnt counts
        // stores and loads together, in order).  The next candidate's entry
        // (SMEM) and moments (VMEM) are fetched one iteration ahead.
        auto sload = [](const int2* p) -> int2 {   // uniform address -> s_load_dwordx2
            const unsigned long long v = *(const __attribute__((address_space(4))) unsigned long long*)p;
            return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
        };
        int2 cur = cb + wave < ce ? sload(t.sorted + cb + wave) : make_int2(0, 0);
        MomEntry mb_cur{0.0, 0u};
        if (cb + wave < ce) {
            const int pk = cur.y, q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
            if (lane < V) mb_cur = load_mom(mom, (r * sc.W + q) * V + lane);
        }
        for (int j = cb + wave; j < ce; j += kT5Waves) {
            const int2 nxt = j + kT5Waves < ce ? sload(t.sorted + j + kT5Waves) : make_int2(0, 0);
            MomEntry mb_nxt{0.0, 0u};
            if (j + kT5Waves < ce) {
                const int pk = nxt.y, q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
                if (lane < V) mb_nxt = load_mom(mom, (r * sc.W + q) * V + lane);
            }
            const int pk = cur.y;
            const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
            const int q0 = q - WID, o = q0 & 3;
            const int k0 = (q0 >> 2) - kq0;
            const MomEntry mb = mb_cur;
            // the reference view's moments: lane R's entry
            const uint32_t ma_sb = __builtin_amdgcn_readlane(mb.sb, R);
            const uint2 wa2 = make_uint2(__builtin_amdgcn_readlane((uint32_t)__double_as_longlong(mb.w), R),
                                         __builtin_amdgcn_readlane((uint32_t)((uint64_t)__double_as_longlong(mb.w) >> 32), R));
            const double wa = __longlong_as_double(((uint64_t)wa2.y << 32) | wa2.x);
            const uint32_t* basep = lds + (r - WID - y0) * RS + k0 * QS + lane;
            // the reference view's quads: same LDS address in every lane (broadcast)
            const uint32_t* refl = basep - lane + R;
            uint32_t Sab = 0;
            if (lane < V) {
                switch (o) {
                    case 0: Sab = sab_rows_stream<WID, 0, RS, QS>(basep, refl); break;
                    case 1: Sab = sab_rows_stream<WID, 1, RS, QS>(basep, refl); break;
                    case 2: Sab = sab_rows_stream<WID, 2, RS, QS>(basep, refl); break;
                    default: Sab = sab_rows_stream<WID, 3, RS, QS>(basep, refl); break;
                }
            }
            // num = n S_ab - S_a S_b (|num| < 2^31 for windows up to 11x11: 24-bit
            // multiplies, exact).  With w = 1/sqrt(n S_bb - S_b^2) per (pixel, view)
            // from the moments table, ctNcc * (n-1) = n num w_a w_b; it is
            // compared with thr (n-1).  The three roundings leave < 2e-15 relative
            // error, so a relative band of 1e-8 around the threshold (far wider
            // than the reference's own rounding) goes to k_score_fix, which
            // decides those lanes with the numpy-order ctNcc.
            static_assert(NPX <= 121, "24-bit moment products need NB <= 11");
            const int32_t num = (int32_t)(__umul24(NPX, Sab) - __umul24(ma_sb, mb.sb));
            const bool live = lane < V && lane != R && mb.w > 0.0 && wa > 0.0;
            bool pass = false, guard = false;
            double ncc = 0.0;
            if (live) {
                if (a.thr >= 0.01) {
                    const double tk = a.thr * (double)(NPX - 1);
                    const double z = ((double)num * ((double)NPX * wa)) * mb.w;   // ncc (n-1)
                    guard = fabs(z - tk) <= 1e-8 * tk;
                    pass = z > tk;
                    ncc = z;
                } else {
                    // the reference view's n S_aa - S_a^2 from its (wave-uniform) w: lane R
                    // itself is not live, so its lane value cannot be read back here
                    const int32_t db = mom_db(mb);
                    const int32_t da = mom_db(MomEntry{wa, 0u});
                    ncc = ((double)num * (double)NPX) /
                          ((double)(NPX - 1) * sqrt((double)da * (double)db));
                    guard = fabs(ncc - a.thr) <= kGuard;
                    pass = ncc > a.thr;
                    ncc *= (double)(NPX - 1);
                }
            }
            if (__ballot(guard) != 0 && lane == 0) t.fix_list[atomicAdd(t.fix_count, 1)] = cur.x;
            const uint64_t m = __ballot(pass);
            const int cnt = __popcll(m);
            double avgv = 0.0;
            if (a.avg && cnt)
                avgv = wave_sum_dpp(pass ? ncc : 0.0) * (c_recip.r[cnt] * (1.0 / (double)(NPX - 1)));
            const int slot = j - cb;
            if (lane == 0) {
                o_mask[slot] = m;
                o_avg[slot] = avgv;
                o_cnt[slot] = cnt;
                o_idx[slot] = cur.x;
            }
            cur = nxt;
            mb_cur = mb_nxt;
        }
        __syncthreads();
        STAMP(2);
        for (int k = threadIdx.x; k < ce - cb; k += blockDim.x) {
            const int i = o_idx[k];
            a.mask[i] = o_mask[k];
            a.count[i] = o_cnt[k];
            if (a.avg) a.avg[i] = o_avg[k];
        }
        __syncthreads();
        STAMP(3);
    }
}


// ---------------------------------------------------------------------------
// Tiled scorer v4 (V <= 64, variant 11, not the default): k_score_tiled3's work split and
// arithmetic, with every window read an 8-byte-aligned ds_read_b64.  On gfx950
// a ds_read_b64 moves 8 B per lane in ~2.7 LDS cycles per wave-instruction,
// a ds_read2_b32 in ~4.4 (tools/ubench/lds_b64.hip), and the LDS pipe bounds
// this kernel.  The region image is kept twice, as pairs of adjacent quads
// [row][pair][view][2 dwords]: pairs (0,1), (2,3), ... in the even image and
// (1,2), (3,4), ... in the odd one, so a window row starting at quad k0 is
// ceil(NQ/2) aligned b64 reads from image (k0 & 1), lane v at dword 2v (64
// banks, no conflict); the reference view's quads are the same reads at lane
// R's address (broadcast).  The doubled image (55 KB at wid 5, V = 48) is
// shared by 8 waves, so two workgroups per CU keep 4 waves per SIMD.
constexpr int kT4Threads = 512, kT4Waves = kT4Threads / 64, kStage4 = 4;

template <int WID>
struct PairGeom {
    using G = TileGeom<WID>;
    // pairs per region row (both images): the largest (k0 >> 1) + ceil(NQ_o / 2)
    // over window byte offsets o and first quads k0 whose window fits the region
    static constexpr int np() {
        int m = 0;
        for (int o = 0; o < 4; ++o) {
            const int nq = (o + G::NB + 3) / 4;
            for (int k0 = 0; k0 + nq <= G::NQ; ++k0) {
                const int v = (k0 >> 1) + (nq + 1) / 2;
                if (v > m) m = v;
            }
        }
        return m;
    }
    // ... and room for every staged quad (even image: pair NQ-1 >> 1)
    static constexpr int NP = np() > (G::NQ + 1) / 2 ? np() : (G::NQ + 1) / 2;
};

template <int WID, int O, int RS, int PS>
DEV uint32_t sab_pairs(const uint32_t* own_g, const uint32_t* ref_g, uint32_t zm) {
    using M = QuadMasks<WID, O>;
    constexpr int NB = 2 * WID + 1;
    constexpr int NPR = (M::NQ + 1) / 2;   // b64 reads per row
    using lds_u64 = __attribute__((address_space(3))) const unsigned long long;
    unsigned long long d[NB][NPR], e[NB][NPR];
#pragma unroll
    for (int p = 0; p < NPR; ++p) {
        lds_u64* o = (lds_u64*)(own_g + p * PS);
        lds_u64* r = (lds_u64*)(ref_g + p * PS);
        asm volatile("" : "+v"(o));
        asm volatile("" : "+v"(r));
#pragma unroll
        for (int row = 0; row < NB; ++row) {
            d[row][p] = o[row * (RS / 2)];
            e[row][p] = r[row * (RS / 2)];
        }
    }
    uint32_t ab[M::NQ];
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) ab[jj] = 0;
#pragma unroll
    for (int row = 0; row < NB; ++row)
#pragma unroll
        for (int jj = 0; jj < M::NQ; ++jj) {
            const uint32_t m = M::mask(jj);
            const uint32_t ev = (uint32_t)(e[row][jj >> 1] >> (32 * (jj & 1)));
            const uint32_t dv = (uint32_t)(d[row][jj >> 1] >> (32 * (jj & 1)));
            const uint32_t am = (m == 0xffffffffu) ? ev : (ev & m);
            ab[jj] = __builtin_amdgcn_udot4(am, dv, ab[jj], false);
        }
    if constexpr (M::NQ & 1) {
        // the last pair's upper quad lies past the window: "use" it (times the
        // opaque zero zm) so the own read stays a ds_read_b64 -- as a
        // ds_read_b32 at lane stride 2 dwords it would take a 2-way bank
        // conflict (~4.2 LDS cycles against ~2.8).  The broadcast side may
        // narrow: same-address reads do not conflict.
#pragma unroll
        for (int row = 0; row < NB; ++row)
            ab[0] = __builtin_amdgcn_udot4(zm, (uint32_t)(d[row][NPR - 1] >> 32), ab[0], false);
    }
    uint32_t sum = 0;
#pragma unroll
    for (int jj = 0; jj < M::NQ; ++jj) sum += ab[jj];
    return sum;
}

template <int WID, int QS>
// no-load-store-opt: the SI load/store optimizer would pair the row reads
// into ds_read2_b64 (8 LDS cycles per 16 B, as slow as ds_read2_b32)
__global__ __launch_bounds__(kT4Threads, 4) __attribute__((target("no-load-store-opt"))) void k_score_tiled4(const SceneDev sc, const ScoreArgs a,
                                                                const TiledArgs t) {
    using G = TileGeom<WID>;
    constexpr int NB = 2 * WID + 1;
    constexpr int NPX = NB * NB;
    constexpr int NP = PairGeom<WID>::NP;
    constexpr int PS = 2 * QS;               // dwords per (row, pair)
    constexpr int RS = NP * PS;              // dwords per region row
    constexpr int IMG = G::ROWS * RS;        // dwords per image
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int V = sc.V;
    const int n_items = t.item_off[t.ntiles];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const MomEntry* __restrict__ mom = sc.mom[WID];
    uint32_t zm = 0;                 // zero the compiler cannot see through (sab_pairs)
    asm volatile("" : "+s"(zm));
    uint64_t* o_mask = (uint64_t*)(lds + 2 * IMG);
    double* o_avg = (double*)(o_mask + t.chunk);
    int32_t* o_cnt = (int32_t*)(o_avg + t.chunk);
    int32_t* o_idx = o_cnt + t.chunk;
    __shared__ int s_item;
    for (;;) {
        if (threadIdx.x == 0) s_item = atomicAdd(&t.tile_count[t.ntiles], 1);
        __syncthreads();
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= n_items) break;
        const unsigned long long itv =
            *(const __attribute__((address_space(4))) unsigned long long*)(t.items + item);
        const int tile = (int)(uint32_t)itv, chunk = (int)(uint32_t)(itv >> 32);
        const int cb = t.tile_off[tile] + chunk * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int y0 = ty * kTH - WID;
        const int kq0 = tx * (kTW / 4) + G::KQ0;
        {
            // one thread per (row, pair, view): quads 2p, 2p+1, 2p+2 of that view
            // (dword loads, consecutive lanes = consecutive views) -> one
            // ds_write_b64 into each image (8 contiguous bytes per lane: no
            // bank conflict)
            const int total = G::ROWS * NP * V;
            for (int base = 0; base < total; base += kStage4 * kT4Threads) {
                uint32_t g[kStage4][3];
                int dst[kStage4];
#pragma unroll
                for (int u = 0; u < kStage4; ++u) {
                    const int k = base + u * kT4Threads + (int)threadIdx.x;
                    dst[u] = -1;
                    g[u][0] = g[u][1] = g[u][2] = 0;
                    if (k < total) {
                        const int rp = k / V, v = k - rp * V;
                        const int ry = rp / NP, pp = rp - ry * NP;
                        const int y = y0 + ry, gq = kq0 + 2 * pp;
                        if (y >= 0 && y < sc.H) {
                            const uint8_t* rowb = sc.stack + (int64_t)y * sc.row_bytes + v * 4;
#pragma unroll
                            for (int h = 0; h < 3; ++h)
                                if (gq + h >= 0 && gq + h < sc.Wq)
                                    g[u][h] = *(const uint32_t*)(rowb + (int64_t)(gq + h) * V * 4);
                        }
                        dst[u] = ry * RS + pp * PS + 2 * v;
                    }
                }
#pragma unroll
                for (int u = 0; u < kStage4; ++u)
                    if (dst[u] >= 0) {
                        *(uint2*)(lds + dst[u]) = make_uint2(g[u][0], g[u][1]);
                        *(uint2*)(lds + IMG + dst[u]) = make_uint2(g[u][1], g[u][2]);
                    }
            }
        }
        __syncthreads();
        auto sload = [](const int2* p) -> int2 {
            const unsigned long long v = *(const __attribute__((address_space(4))) unsigned long long*)p;
            return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
        };
        int2 cur = cb + wave < ce ? sload(t.sorted + cb + wave) : make_int2(0, 0);
        MomEntry mb_cur{0.0, 0u};
        if (cb + wave < ce) {
            const int pk = cur.y, q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
            if (lane < V) mb_cur = load_mom(mom, (r * sc.W + q) * V + lane);
        }
        for (int j = cb + wave; j < ce; j += kT4Waves) {
            const int2 nxt = j + kT4Waves < ce ? sload(t.sorted + j + kT4Waves) : make_int2(0, 0);
            MomEntry mb_nxt{0.0, 0u};
            if (j + kT4Waves < ce) {
                const int pk = nxt.y, q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
                if (lane < V) mb_nxt = load_mom(mom, (r * sc.W + q) * V + lane);
            }
            const int pk = cur.y;
            const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
            const int q0 = q - WID, o = q0 & 3;
            const int k0 = (q0 >> 2) - kq0;
            const MomEntry mb = mb_cur;
            const uint32_t ma_sb = __builtin_amdgcn_readlane(mb.sb, R);
            const uint2 wa2 = make_uint2(__builtin_amdgcn_readlane((uint32_t)__double_as_longlong(mb.w), R),
                                         __builtin_amdgcn_readlane((uint32_t)((uint64_t)__double_as_longlong(mb.w) >> 32), R));
            const double wa = __longlong_as_double(((uint64_t)wa2.y << 32) | wa2.x);
            // image (k0 & 1), pair k0 >> 1, lane's view at dword 2 * lane
            const uint32_t* rowp = lds + (k0 & 1) * IMG + (r - WID - y0) * RS + (k0 >> 1) * PS;
            const uint32_t* basep = rowp + 2 * lane;
            const uint32_t* refl = rowp + 2 * R;
            uint32_t Sab = 0;
            if (lane < V) {
                switch (o) {
                    case 0: Sab = sab_pairs<WID, 0, RS, PS>(basep, refl, zm); break;
                    case 1: Sab = sab_pairs<WID, 1, RS, PS>(basep, refl, zm); break;
                    case 2: Sab = sab_pairs<WID, 2, RS, PS>(basep, refl, zm); break;
                    default: Sab = sab_pairs<WID, 3, RS, PS>(basep, refl, zm); break;
                }
            }
            // decision: as k_score_tiled3 (see there)
            const int32_t num = (int32_t)(__umul24(NPX, Sab) - __umul24(ma_sb, mb.sb));
            const bool live = lane < V && lane != R && mb.w > 0.0 && wa > 0.0;
            bool pass = false, guard = false;
            double ncc = 0.0;
            if (live) {
                if (a.thr >= 0.01) {
                    const double tk = a.thr * (double)(NPX - 1);
                    const double z = ((double)num * ((double)NPX * wa)) * mb.w;
                    guard = fabs(z - tk) <= 1e-8 * tk;
                    pass = z > tk;
                    ncc = z;
                } else {
                    const int32_t db = mom_db(mb);
                    const int32_t da = mom_db(MomEntry{wa, 0u});
                    ncc = ((double)num * (double)NPX) /
                          ((double)(NPX - 1) * sqrt((double)da * (double)db));
                    guard = fabs(ncc - a.thr) <= kGuard;
                    pass = ncc > a.thr;
                    ncc *= (double)(NPX - 1);
                }
            }
            if (__ballot(guard) != 0 && lane == 0) t.fix_list[atomicAdd(t.fix_count, 1)] = cur.x;
            const uint64_t m = __ballot(pass);
            const int cnt = __popcll(m);
            double avgv = 0.0;
            if (a.avg && cnt)
                avgv = wave_sum_dpp(pass ? ncc : 0.0) * (c_recip.r[cnt] * (1.0 / (double)(NPX - 1)));
            const int slot = j - cb;
            if (lane == 0) {
                o_mask[slot] = m;
                o_avg[slot] = avgv;
                o_cnt[slot] = cnt;
                o_idx[slot] = cur.x;
            }
            cur = nxt;
            mb_cur = mb_nxt;
        }
        __syncthreads();
        for (int k = threadIdx.x; k < ce - cb; k += blockDim.x) {
            const int i = o_idx[k];
            a.mask[i] = o_mask[k];
            a.count[i] = o_cnt[k];
            if (a.avg) a.avg[i] = o_avg[k];
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Tiled scorer for V > 64 (256 views): the views are
// split into groups of 64 and a work item is (tile chunk, view group).  The
// workgroup stages the tile's window region of its 64 views only
// ([row][quad][64] dwords, 36.9 KB at wid 5), one lane per view of the group
// as in k_score_tiled3.  The reference view R is generally in another group,
// so each wave copies the current candidate's 11x4 reference quads from the
// view-major copy gv into a private LDS slot (one dword per lane, prefetched one
// candidate ahead) and reads them from there as broadcasts.  (Masking the
// slot once instead of per lane measured 12 % slower: 2.96 vs 2.65 ms.)  A group writes
// its own mask word (64 views = one word) and a partial (count, sum of
// ncc*(n-1)); k_group_finalize adds the partials.
// ---------------------------------------------------------------------------
constexpr int kTGThreads = 256, kTGWaves = kTGThreads / 64;

template <int WID>
__global__ __launch_bounds__(kTGThreads, 3) void k_score_tiledg(const SceneDev sc, const ScoreArgs a,
                                                                const TiledArgs t) {
    using G = TileGeom<WID>;
    constexpr int NB = 2 * WID + 1;
    constexpr int NPX = NB * NB;
    constexpr int QS = 64;
    constexpr int RS = G::NQ * QS;
    constexpr int SLOT = NB * 4;                 // reference quads per wave: [row][4]
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int V = sc.V;
    const int NG = t.groups;
    // XCD-aware work queues: blocks b and b + 8 share an XCD (and its L2), so
    // queue x = blockIdx % 8 hands out the chunks c = x (mod 8), all NG view
    // groups of a chunk in a row: the groups of one chunk run on one XCD and
    // share its L2 lines (candidate list, reference rows of gv).
    const int xq = blockIdx.x & 7;
    const int n_chunks = t.item_off[t.ntiles];
    const int n_items = n_chunks > xq ? ((n_chunks - xq + 7) >> 3) * NG : 0;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const MomEntry* __restrict__ mom = sc.mom[WID];
    uint64_t* o_mask = (uint64_t*)(lds + G::ROWS * RS);
    double* o_sum = (double*)(o_mask + t.chunk);
    int32_t* o_cnt = (int32_t*)(o_sum + t.chunk);
    int32_t* o_idx = o_cnt + t.chunk;
    uint32_t* slot = (uint32_t*)(o_idx + t.chunk) + wave * SLOT;
    __shared__ int s_item;
    // the reference quads of candidate pk (lanes < SLOT), from the view-major
    // copy gv: a window row's 4 quads are 16 contiguous bytes there (one cache
    // line per row instead of one per quad in the view-interleaved stack);
    // the row pitch Wp >= 4 (W/4 + 1) keeps the last quad in bounds
    auto ref_quads = [&](int pk) -> uint32_t {
        uint32_t v = 0;
        if (lane < SLOT) {
            const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
            const int row = lane >> 2, gq = ((q - WID) >> 2) + (lane & 3);
            v = *(const uint32_t*)(sc.gv + ((int64_t)R * sc.H + (r - WID + row)) * sc.Wp + 4 * gq);
        }
        return v;
    };
    for (;;) {
        if (threadIdx.x == 0) s_item = atomicAdd(&t.xq[xq], 1);
        __syncthreads();
        const int k = __builtin_amdgcn_readfirstlane(s_item);
        if (k >= n_items) break;
        const int kc = k / NG, g = k - kc * NG;
        const int item = xq + 8 * kc;
        const int vb = 64 * g, nv = min(64, V - vb);
        const unsigned long long itv =
            *(const __attribute__((address_space(4))) unsigned long long*)(t.items + item);
        const int tile = (int)(uint32_t)itv, chunk = (int)(uint32_t)(itv >> 32);
        const int cb = t.tile_off[tile] + chunk * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int y0 = ty * kTH - WID;
        const int kq0 = tx * (kTW / 4) + G::KQ0;
        {
            const int cpq = nv >> 2, cpr = G::NQ * cpq, total = G::ROWS * cpr;
            for (int base = 0; base < total; base += 8 * kTGThreads) {
                uint4 buf[8];
                int dst[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int k = base + u * kTGThreads + (int)threadIdx.x;
                    dst[u] = -1;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (k < total) {
                        const int ry = k / cpr, rem = k - ry * cpr;
                        const int kq = rem / cpq, vq = rem - kq * cpq;
                        const int y = y0 + ry, gq = kq0 + kq;
                        if (y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                            buf[u] = *(const uint4*)(sc.stack + (int64_t)y * sc.row_bytes +
                                                      (int64_t)gq * V * 4 + (vb + 4 * vq) * 4);
                        dst[u] = (ry * G::NQ + kq) * QS + vq * 4;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (dst[u] >= 0) *(uint4*)(lds + dst[u]) = buf[u];
            }
        }
        auto sload = [](const int2* p) -> int2 {
            const unsigned long long v = *(const __attribute__((address_space(4))) unsigned long long*)p;
            return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
        };
        auto pix = [&](int pk) -> int64_t { return (int64_t)((pk >> 11) & 0x7ff) * sc.W + (pk & 0x7ff); };
        int2 cur = cb + wave < ce ? sload(t.sorted + cb + wave) : make_int2(0, 0);
        MomEntry mb_cur{0.0, 0u}, ma_cur{0.0, 0u};
        if (cb + wave < ce) {
            if (lane < nv) mb_cur = load_mom(mom, pix(cur.y) * V + vb + lane);
            ma_cur = load_mom(mom, pix(cur.y) * V + ((cur.y >> 22) & 0x3ff));
            const uint32_t rq = ref_quads(cur.y);
            if (lane < SLOT) slot[lane] = rq;
        }
        __syncthreads();   // region image complete
        for (int j = cb + wave; j < ce; j += kTGWaves) {
            const bool more = j + kTGWaves < ce;
            const int2 nxt = more ? sload(t.sorted + j + kTGWaves) : make_int2(0, 0);
            MomEntry mb_nxt{0.0, 0u}, ma_nxt{0.0, 0u};
            uint32_t rq_nxt = 0;
            if (more) {
                if (lane < nv) mb_nxt = load_mom(mom, pix(nxt.y) * V + vb + lane);
                ma_nxt = load_mom(mom, pix(nxt.y) * V + ((nxt.y >> 22) & 0x3ff));
                rq_nxt = ref_quads(nxt.y);
            }
            const int pk = cur.y;
            const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
            const int q0 = q - WID, o = q0 & 3;
            const int k0 = (q0 >> 2) - kq0;
            const MomEntry mb = mb_cur, ma = ma_cur;
            const uint32_t* basep = lds + (r - WID - y0) * RS + k0 * QS + lane;
            uint32_t Sab = 0;
            if (lane < nv) {
                switch (o) {
                    case 0: Sab = sab_rows<WID, 0, RS, QS, 4, 1>(basep, slot); break;
                    case 1: Sab = sab_rows<WID, 1, RS, QS, 4, 1>(basep, slot); break;
                    case 2: Sab = sab_rows<WID, 2, RS, QS, 4, 1>(basep, slot); break;
                    default: Sab = sab_rows<WID, 3, RS, QS, 4, 1>(basep, slot); break;
                }
            }
            // the next candidate's reference quads replace this one's: the wave's
            // LDS operations complete in program order, after the reads above
            if (more && lane < SLOT) slot[lane] = rq_nxt;
            const int32_t num = (int32_t)(__umul24(NPX, Sab) - __umul24(ma.sb, mb.sb));
            const bool live = lane < nv && vb + lane != R && mb.w > 0.0 && ma.w > 0.0;
            bool pass = false, guard = false;
            double ncc = 0.0;
            if (live) {
                if (a.thr >= 0.01) {
                    const double tk = a.thr * (double)(NPX - 1);
                    const double z = ((double)num * ((double)NPX * ma.w)) * mb.w;
                    guard = fabs(z - tk) <= 1e-8 * tk;
                    pass = z > tk;
                    ncc = z;
                } else {
                    const int32_t db = mom_db(mb), da = mom_db(ma);
                    ncc = ((double)num * (double)NPX) /
                          ((double)(NPX - 1) * sqrt((double)da * (double)db));
                    guard = fabs(ncc - a.thr) <= kGuard;
                    pass = ncc > a.thr;
                    ncc *= (double)(NPX - 1);
                }
            }
            if (__ballot(guard) != 0 && lane == 0) t.fix_list[atomicAdd(t.fix_count, 1)] = cur.x;
            const uint64_t m = __ballot(pass);
            const int cnt = __popcll(m);
            const double sum = (a.avg && cnt) ? wave_sum_dpp(pass ? ncc : 0.0) : 0.0;
            const int sl = j - cb;
            if (lane == 0) {
                o_mask[sl] = m;
                o_sum[sl] = sum;
                o_cnt[sl] = cnt;
                o_idx[sl] = cur.x;
            }
            cur = nxt;
            mb_cur = mb_nxt;
            ma_cur = ma_nxt;
        }
        __syncthreads();
        const int words = (V + 63) >> 6;
        for (int k = threadIdx.x; k < ce - cb; k += blockDim.x) {
            const int64_t i = o_idx[k];
            a.mask[i * words + g] = o_mask[k];
            t.part_cnt[i * NG + g] = o_cnt[k];
            t.part_sum[i * NG + g] = o_sum[k];
        }
        __syncthreads();
    }
}

// count and avg_ncc_score of every scored candidate from its view groups'
// partials (same scaling as k_score_tiled3: sum * (1/cnt) * (1/(n-1)))
__global__ void k_group_finalize(const ScoreArgs a, const TiledArgs t, int npx) {
    const int NG = t.groups;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (t.cand_key[i] < 0) continue;     // invalid window: k_bin wrote the outputs
        int cnt = 0;
        double sum = 0.0;
        for (int g = 0; g < NG; ++g) {
            cnt += t.part_cnt[i * NG + g];
            sum += t.part_sum[i * NG + g];
        }
        a.count[i] = cnt;
        if (a.avg) a.avg[i] = cnt ? sum * ((1.0 / (double)cnt) * (1.0 / (double)(npx - 1))) : 0.0;
    }
}

// ---------------------------------------------------------------------------
// MFMA scorer.  S_ab of a candidate (pixel p, reference view R) against every
// view v is a box sum over the window of the product image g_R * g_v.  For one
// 16x16-pixel output tile and one R, all of them -- 16 x-positions x every
// view x every output row -- come from one chain of
// v_mfma_i32_16x16x64_i8 per 16-view slice: row y of the tile region
// contributes  A_y(x, k) . B_y(k, v)  with A_y = g_R(y, k) masked to the band
// x <= k - off0 <= x + 2 WID (the window's columns for output x) and
// B_y = g_v(y, k); a running prefix over rows gives the vertical window sum
// S_j = C_{j+2WID} - C_{j-1}.  Pixels are stored as g - 128 (signed bytes,
// exact): sum (g_a-128)(g_b-128) = S_ab - 128 (S_a + S_b) + 16384 n.
// Per candidate only the decision epilogue (moments, squared comparison,
// avg) remains on the VALU, one lane per view as in k_score_tiled3.
// ---------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kMTW = 16, kMTH = 16;          // output tile (x, y)
constexpr int kMThreads = 512, kMWaves = kMThreads / 64;
constexpr int kMChunk = 1024;                // candidates per work item
constexpr int kMNB = 16;                     // candidates per R pass (per-wave S buffer)

template <int WID, int NT>
struct MfmaGeom {
    static constexpr int NB = 2 * WID + 1;
    static constexpr int NR = kMTH + 2 * WID;     // region rows
    static constexpr int VS = NR * 32 + 16;       // bytes per view: an odd number of 16-B units
    static constexpr int NV = NT * 16;            // view slots
    static constexpr int NKEY = 64 * kMTH;        // (R, output row) sort keys, V <= 64
    static constexpr int OFF0 = (4 - WID % 4) % 4;   // window column of output x = x + OFF0
    static_assert(kMTW + OFF0 + 2 * WID <= 32, "window must fit the 32 region columns");
    static constexpr int O_REG = 0;
    static constexpr int O_CU = (NV * VS + 15) / 16 * 16;             // int2[kMChunk] tile order
    static constexpr int O_CS = O_CU + 8 * kMChunk;                    // int2[kMChunk] key order
    static constexpr int O_HS = O_CS + 8 * kMChunk;                    // int[NKEY + 1] key starts
    static constexpr int O_CUR = O_HS + 4 * (NKEY + 4);                // int[NKEY] counts/cursors
    static constexpr int O_SB = O_CUR + 4 * NKEY;                      // int[waves][kMNB][64]
    static constexpr int O_OM = O_SB + 4 * kMWaves * kMNB * 64;        // u64[kMChunk]
    static constexpr int O_OA = O_OM + 8 * kMChunk;                    // double[kMChunk]
    static constexpr int O_OC = O_OA + 8 * kMChunk;                    // int[kMChunk]
    static constexpr int O_WT = O_OC + 4 * kMChunk;                    // int[kMWaves]
    static constexpr int BYTES = O_WT + 4 * kMWaves;
};

template <int WID, int NT>
__global__ __launch_bounds__(kMThreads, 2) void k_score_mfma(const SceneDev sc, const ScoreArgs a,
                                                             const TiledArgs t) {
    using G = MfmaGeom<WID, NT>;
    constexpr int NB = G::NB, NPX = NB * NB, NR = G::NR, VS = G::VS;
    constexpr int RING = NB + 1;              // prefixes C_{y-NB} .. C_y
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* reg = smem + G::O_REG;
    int2* cu = (int2*)(smem + G::O_CU);
    int2* cs = (int2*)(smem + G::O_CS);
    int* hs = (int*)(smem + G::O_HS);
    int* cur = (int*)(smem + G::O_CUR);
    int* sbuf = (int*)(smem + G::O_SB);
    uint64_t* o_mask = (uint64_t*)(smem + G::O_OM);
    double* o_avg = (double*)(smem + G::O_OA);
    int32_t* o_cnt = (int32_t*)(smem + G::O_OC);
    int* wt = (int*)(smem + G::O_WT);
    __shared__ int s_item;

    const int V = sc.V;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n_items = t.item_off[t.ntiles];
    const int nkey = V * kMTH;
    const MomEntry* __restrict__ mom = sc.mom[WID];
    const int lx = lane & 15, lh = lane >> 4;
    // A-fragment band mask of this lane: output x = lx, region columns 16 lh + b
    uint32_t bm[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int col = 16 * lh + 4 * d + b;
            if (lh < 2 && col >= lx + G::OFF0 && col <= lx + G::OFF0 + 2 * WID) m |= 0xffu << (8 * b);
        }
        bm[d] = m;
    }
    int* my_sb = sbuf + wave * kMNB * 64;
#ifdef MVS_STAMPS
    unsigned long long st_prev = 0;
#endif

    for (;;) {
        if (tid == 0) s_item = atomicAdd(&t.tile_count[t.ntiles], 1);
        __syncthreads();
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= n_items) break;
        STAMP(0);
        int lo = 0, hi = t.ntiles;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (t.item_off[mid] <= item) lo = mid; else hi = mid;
        }
        const int tile = lo;
        const int cb = t.tile_off[tile] + (item - t.item_off[tile]) * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int nc = ce - cb;
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int x0 = tx * kMTW, yo0 = ty * kMTH;
        const int y0 = yo0 - WID;
        const int kq0 = (x0 - WID) >> 2;          // floor
        // ---- stage the region: NR rows x 8 quads x all views, as g ^ 0x80 ----
        {
            const int cpq = V >> 2, cpr = 8 * cpq, total = NR * cpr;
            for (int base = 0; base < total; base += 4 * kMThreads) {
                uint4 buf[4];
                int dst[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = base + u * kMThreads + tid;
                    dst[u] = -1;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (k < total) {
                        const int ry = k / cpr, rem = k - ry * cpr;
                        const int kq = rem / cpq, vq = rem - kq * cpq;
                        const int y = y0 + ry, gq = kq0 + kq;
                        if (y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                            buf[u] = *(const uint4*)(sc.stack + (int64_t)y * sc.row_bytes +
                                                      (int64_t)gq * V * 4 + vq * 16);
                        dst[u] = (4 * vq) * VS + ry * 32 + kq * 4;
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (dst[u] >= 0) {
                        uint8_t* d = reg + dst[u];
                        *(uint32_t*)(d) = buf[u].x ^ 0x80808080u;
                        *(uint32_t*)(d + VS) = buf[u].y ^ 0x80808080u;
                        *(uint32_t*)(d + 2 * VS) = buf[u].z ^ 0x80808080u;
                        *(uint32_t*)(d + 3 * VS) = buf[u].w ^ 0x80808080u;
                    }
            }
        }
        // ---- candidates of the item, counting-sorted by (R, output row) ----
        for (int k = tid; k < nkey; k += kMThreads) cur[k] = 0;
        __syncthreads();
        for (int k = tid; k < nc; k += kMThreads) {
            const int2 e = t.sorted[cb + k];
            cu[k] = e;
            const int r = (e.y >> 11) & 0x7ff, R = (e.y >> 22) & 0x3ff;
            atomicAdd(&cur[R * kMTH + (r - yo0)], 1);
        }
        __syncthreads();
        {   // exclusive scan of cur[0 .. nkey) into hs (two keys per thread)
            const int b = 2 * tid;
            const int c0 = b < nkey ? cur[b] : 0, c1 = b + 1 < nkey ? cur[b + 1] : 0;
            int sum = c0 + c1;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int u = __shfl_up(sum, off, 64);
                if (lane >= off) sum += u;
            }
            if (lane == 63) wt[wave] = sum;
            __syncthreads();
            int before = 0;
            for (int w = 0; w < wave; ++w) before += wt[w];
            const int excl = before + sum - (c0 + c1);
            if (b < nkey) { hs[b] = excl; cur[b] = excl; }
            if (b + 1 < nkey) { hs[b + 1] = excl + c0; cur[b + 1] = excl + c0; }
            if (tid == kMThreads - 1) hs[nkey] = before + sum;
        }
        __syncthreads();
        for (int k = tid; k < nc; k += kMThreads) {
            const int2 e = cu[k];
            const int r = (e.y >> 11) & 0x7ff, R = (e.y >> 22) & 0x3ff;
            cs[atomicAdd(&cur[R * kMTH + (r - yo0)], 1)] = e;
        }
        __syncthreads();
        STAMP(1);
        // ---- one reference view per wave at a time ----
        for (int R = wave; R < V; R += kMWaves) {
            const int gb = __builtin_amdgcn_readfirstlane(hs[R * kMTH]);
            const int ge = __builtin_amdgcn_readfirstlane(hs[(R + 1) * kMTH]);
            for (int pb = gb; pb < ge; pb += kMNB) {
                const int pe = min(pb + kMNB, ge);
                STAMP_T(tp0);
                // moments of the pass's candidates, in flight during the MFMA rows
                uint2 mbs[kMNB];
#pragma unroll
                for (int c = 0; c < kMNB; ++c) {
                    mbs[c] = make_uint2(0, 0);
                    if (pb + c < pe && lane < V) {
                        const int pk = cs[pb + c].y;
                        const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff;
                        { const MomEntry me = load_mom(mom, (r * sc.W + q) * V + lane);
                          mbs[c] = make_uint2(me.sb, (uint32_t)(((int64_t)mom_db(me) + (int64_t)me.sb * me.sb) / NPX)); }
                    }
                }
                // MFMA rows: ring of prefixes C_y over the region rows
                const uint8_t* ra = reg + R * VS + 16 * (lh & 1);
                v4i C[RING][NT];
#pragma unroll
                for (int y = 0; y < NR; ++y) {
                    const uint4 av = *(const uint4*)(ra + y * 32);
                    const v4i A = {(int)(av.x & bm[0]), (int)(av.y & bm[1]), (int)(av.z & bm[2]),
                                   (int)(av.w & bm[3])};
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        const uint4 bv = *(const uint4*)(reg + (16 * nt + lx) * VS + y * 32 + 16 * (lh & 1));
                        const v4i B = {(int)bv.x, (int)bv.y, (int)bv.z, (int)bv.w};
                        const v4i zero = {0, 0, 0, 0};
                        C[y % RING][nt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                            A, B, y == 0 ? zero : C[(y + RING - 1) % RING][nt], 0, 0, 0);
                    }
                    if (y >= 2 * WID) {
                        const int j = y - 2 * WID;   // output row
                        const int kb = max(pb, __builtin_amdgcn_readfirstlane(hs[R * kMTH + j]));
                        const int ke = min(pe, __builtin_amdgcn_readfirstlane(hs[R * kMTH + j + 1]));
                        if (kb < ke) {
                            v4i S[NT];
#pragma unroll
                            for (int nt = 0; nt < NT; ++nt)
                                S[nt] = j == 0 ? C[y % RING][nt]
                                               : C[y % RING][nt] - C[(y + 1) % RING][nt];  // C_{j-1} = C_{y-NB}
                            for (int k = kb; k < ke; ++k) {
                                const int pk = __builtin_amdgcn_readfirstlane(cs[k].y);
                                const int x = (pk & 0x7ff) - x0;
                                const int xi = x & 3;
                                if (lh == (x >> 2)) {
                                    int* d = my_sb + (k - pb) * 64 + lx;
#pragma unroll
                                    for (int nt = 0; nt < NT; ++nt) {
                                        const int val = xi == 0 ? S[nt][0] : xi == 1 ? S[nt][1]
                                                      : xi == 2 ? S[nt][2] : S[nt][3];
                                        d[16 * nt] = val;
                                    }
                                }
                            }
                        }
                    }
                }
                STAMP_T(tp1);
                STAMP_ADD(4, tp0, tp1);
                // decision epilogue: one lane per view, as k_score_tiled3
                for (int k = pb; k < pe; ++k) {
                    const int2 e = cs[k];
                    const int ci = __builtin_amdgcn_readfirstlane(e.x);
                    (void)ci;
                    uint2 mb = mbs[0];
#pragma unroll
                    for (int c = 1; c < kMNB; ++c) mb = (k - pb == c) ? mbs[c] : mb;
                    const uint2 ma = make_uint2(__builtin_amdgcn_readlane(mb.x, R),
                                                __builtin_amdgcn_readlane(mb.y, R));
                    const int sab_s = my_sb[(k - pb) * 64 + lane];
                    const uint32_t Sab = (uint32_t)(sab_s + 128 * (int)(ma.x + mb.x) - 16384 * NPX);
                    const int32_t da = (int32_t)(__umul24(NPX, ma.y) - __umul24(ma.x, ma.x));
                    const int32_t db = (int32_t)(__umul24(NPX, mb.y) - __umul24(mb.x, mb.x));
                    const int32_t num = (int32_t)(__umul24(NPX, Sab) - __umul24(ma.x, mb.x));
                    const bool live = lane < V && lane != R && da > 0 && db > 0;
                    bool pass = false, guard = false;
                    double ncc = 0.0;
                    if (live) {
                        if (a.thr >= 0.01) {
                            const double L = (double)num * (double)NPX;
                            if (L > 0.0) {
                                const double tk = a.thr * (double)(NPX - 1);
                                const double rhs = (tk * tk) * ((double)da * (double)db);
                                const double diff = L * L - rhs;
                                guard = fabs(diff) <= 1e-8 * rhs;
                                pass = diff > 0.0;
                                if (pass && a.avg) {
                                    const double D = (double)da * (double)db;
                                    double yv = __builtin_amdgcn_rsq(D);
                                    yv = yv * (1.5 - 0.5 * D * yv * yv);
                                    yv = yv * (1.5 - 0.5 * D * yv * yv);
                                    ncc = L * yv * (1.0 / (double)(NPX - 1));
                                }
                            }
                        } else {
                            ncc = ((double)num * (double)NPX) /
                                  ((double)(NPX - 1) * sqrt((double)da * (double)db));
                            guard = fabs(ncc - a.thr) <= kGuard;
                            pass = ncc > a.thr;
                        }
                    }
                    if (__ballot(guard) != 0 && lane == 0)
                        t.fix_list[atomicAdd(t.fix_count, 1)] = e.x;
                    const uint64_t m = __ballot(pass);
                    const int cnt = __popcll(m);
                    double avgv = 0.0;
                    if (a.avg && cnt) avgv = wave_sum_dpp(pass ? ncc : 0.0) * c_recip.r[cnt];
                    if (lane == 0) {
                        o_mask[k] = m;
                        o_avg[k] = avgv;
                        o_cnt[k] = cnt;
                    }
                }
                STAMP_T(tp2);
                STAMP_ADD(5, tp1, tp2);
                STAMP_ADD(6, 0, (unsigned long long)(pe - pb));
            }
        }
        __syncthreads();
        STAMP(2);
        for (int k = tid; k < nc; k += kMThreads) {
            const int i = cs[k].x;
            a.mask[i] = o_mask[k];
            a.count[i] = o_cnt[k];
            if (a.avg) a.avg[i] = o_avg[k];
        }
        __syncthreads();
        STAMP(3);
    }
}


// ---------------------------------------------------------------------------
// MFMA scorer, v2 (variant 9): same 16x8 tiles and work items as
// k_score_tiled3; per (tile, reference view R) the S_ab sums of every output
// pixel against every view come from v_mfma_i32_16x16x32_i8 chains, one
// 16-view slice at a time:  C_y = A_y . B_y + C_{y-1}  over the 8 + 2 WID
// region rows, A_y(x, k) = g_R(y, k) - 128 masked to the window columns of
// output x (k = 32 region columns = the MFMA's K), B_y(k, v) = g_v(y, k) - 128;
// S(output row j) = C_{j+2WID} - C_{j-1}.  Only the S values of the item's
// candidates are kept (per-wave LDS buffer); the decision epilogue is
// k_score_tiled3's.  Operand bytes per MFMA: 512 (B) + 512 (A, LDS
// broadcast), against ~15 KB of LDS reads per candidate in tiled3.
// ---------------------------------------------------------------------------
typedef long v1l;
constexpr int kM2Threads = 256, kM2Waves = kM2Threads / 64;
constexpr int kM2NB = 16;                    // candidates per R pass

template <int WID, int NT>
struct Mfma2Geom {
    static constexpr int NB = 2 * WID + 1;
    static constexpr int NR = kTH + 2 * WID;        // region rows
    static constexpr int VS = NR * 32 + 8;          // bytes per view: an odd number of 8-B units
    static constexpr int NV = NT * 16;
    static constexpr int NKEY = 64 * kTH;           // (R, output row), V <= 64
    static constexpr int OFF0 = (4 - WID % 4) % 4;  // region column of output x's window = x + OFF0
    static_assert(kTW + OFF0 + 2 * WID <= 32, "window must fit the 32 region columns");
    static constexpr int O_REG = 0;
    static constexpr int O_CS = (NV * VS + 15) / 16 * 16;              // int2[kM2Threads]
    static constexpr int O_HS = O_CS + 8 * kM2Threads;                  // int[NKEY + 4]
    static constexpr int O_CUR = O_HS + 4 * (NKEY + 4);                // int[NKEY]
    static constexpr int O_SB = O_CUR + 4 * NKEY;                      // int[waves][kM2NB][NV]
    static constexpr int O_OM = O_SB + 4 * kM2Waves * kM2NB * NV;      // u64[kM2Threads]
    static constexpr int O_OA = O_OM + 8 * kM2Threads;                 // double[kM2Threads]
    static constexpr int O_OC = O_OA + 8 * kM2Threads;                 // int[kM2Threads]
    static constexpr int O_WT = O_OC + 4 * kM2Threads;                 // int[waves]
    static constexpr int BYTES = O_WT + 4 * kM2Waves;
};

template <int WID, int NT>
__global__ __launch_bounds__(kM2Threads, 3) void k_score_mfma2(const SceneDev sc, const ScoreArgs a,
                                                               const TiledArgs t) {
    using G = Mfma2Geom<WID, NT>;
    constexpr int NB = G::NB, NPX = NB * NB, NR = G::NR, VS = G::VS, NV = G::NV;
    constexpr int RING = NB + 1;              // prefixes C_{y-NB} .. C_y
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint8_t* reg = smem + G::O_REG;
    int2* cs = (int2*)(smem + G::O_CS);
    int* hs = (int*)(smem + G::O_HS);
    int* cur = (int*)(smem + G::O_CUR);
    int* sbuf = (int*)(smem + G::O_SB);
    uint64_t* o_mask = (uint64_t*)(smem + G::O_OM);
    double* o_avg = (double*)(smem + G::O_OA);
    int32_t* o_cnt = (int32_t*)(smem + G::O_OC);
    int* wt = (int*)(smem + G::O_WT);
    __shared__ int s_item;

    const int V = sc.V;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n_items = t.item_off[t.ntiles];
    const int nkey = V * kTH;
    const MomEntry* __restrict__ mom = sc.mom[WID];
    const int lx = lane & 15, lh = lane >> 4;
    // A-operand band mask of this lane: output x = lx, region columns 8 lh + b
    uint32_t bm[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int col = 8 * lh + 4 * d + b;
            if (col >= lx + G::OFF0 && col <= lx + G::OFF0 + 2 * WID) m |= 0xffu << (8 * b);
        }
        bm[d] = m;
    }
    int* my_sb = sbuf + wave * kM2NB * NV;
#ifdef MVS_STAMPS
    unsigned long long st_prev = 0;
#endif

    for (;;) {
        if (tid == 0) s_item = atomicAdd(&t.tile_count[t.ntiles], 1);
        __syncthreads();
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item >= n_items) break;
        STAMP(0);
        int lo = 0, hi = t.ntiles;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (t.item_off[mid] <= item) lo = mid; else hi = mid;
        }
        const int tile = lo;
        const int cb = t.tile_off[tile] + (item - t.item_off[tile]) * t.chunk;
        const int ce = min(cb + t.chunk, t.tile_off[tile + 1]);
        const int nc = ce - cb;                 // <= kM2Threads
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int x0 = tx * kTW, yo0 = ty * kTH;
        const int y0 = yo0 - WID;
        const int kq0 = (x0 - WID) >> 2;        // floor
        // ---- stage the region (NR rows x 8 quads x all views) as g ^ 0x80 ----
        {
            const int cpq = V >> 2, cpr = 8 * cpq, total = NR * cpr;
            for (int base = 0; base < total; base += 4 * kM2Threads) {
                uint4 buf[4];
                int dst[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = base + u * kM2Threads + tid;
                    dst[u] = -1;
                    buf[u] = make_uint4(0, 0, 0, 0);
                    if (k < total) {
                        const int ry = k / cpr, rem = k - ry * cpr;
                        const int kq = rem / cpq, vq = rem - kq * cpq;
                        const int y = y0 + ry, gq = kq0 + kq;
                        if (y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                            buf[u] = *(const uint4*)(sc.stack + (int64_t)y * sc.row_bytes +
                                                      (int64_t)gq * V * 4 + vq * 16);
                        dst[u] = (4 * vq) * VS + ry * 32 + kq * 4;
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (dst[u] >= 0) {
                        uint8_t* d = smem + G::O_REG + dst[u];
                        *(uint32_t*)(d) = buf[u].x ^ 0x80808080u;
                        *(uint32_t*)(d + VS) = buf[u].y ^ 0x80808080u;
                        *(uint32_t*)(d + 2 * VS) = buf[u].z ^ 0x80808080u;
                        *(uint32_t*)(d + 3 * VS) = buf[u].w ^ 0x80808080u;
                    }
            }
        }
        // ---- the item's candidates (one per thread), counting-sorted by (R, row) ----
        for (int k = tid; k < nkey; k += kM2Threads) cur[k] = 0;
        __syncthreads();
        int2 e = make_int2(0, 0);
        int key = -1;
        if (tid < nc) {
            e = t.sorted[cb + tid];
            const int r = (e.y >> 11) & 0x7ff, R = (e.y >> 22) & 0x3ff;
            key = R * kTH + (r - yo0);
            atomicAdd(&cur[key], 1);
        }
        __syncthreads();
        {   // exclusive scan of cur[0 .. nkey) into hs (two keys per thread)
            const int b = 2 * tid;
            const int c0 = b < nkey ? cur[b] : 0, c1 = b + 1 < nkey ? cur[b + 1] : 0;
            int sum = c0 + c1;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int u = __shfl_up(sum, off, 64);
                if (lane >= off) sum += u;
            }
            if (lane == 63) wt[wave] = sum;
            __syncthreads();
            int before = 0;
            for (int w = 0; w < wave; ++w) before += wt[w];
            const int excl = before + sum - (c0 + c1);
            if (b < nkey) { hs[b] = excl; cur[b] = excl; }
            if (b + 1 < nkey) { hs[b + 1] = excl + c0; cur[b + 1] = excl + c0; }
            if (tid == kM2Threads - 1) hs[nkey] = before + sum;
        }
        __syncthreads();
        if (key >= 0) cs[atomicAdd(&cur[key], 1)] = e;
        __syncthreads();
        STAMP(1);
        // ---- one reference view per wave at a time ----
        for (int R = wave; R < V; R += kM2Waves) {
            const int gb = __builtin_amdgcn_readfirstlane(hs[R * kTH]);
            const int ge = __builtin_amdgcn_readfirstlane(hs[(R + 1) * kTH]);
            for (int pb = gb; pb < ge; pb += kM2NB) {
                const int np = min(kM2NB, ge - pb);
                STAMP_T(tp0);
                // the pass's candidates: lane c holds candidate pb + c's packed
                // (q, r, R); their moments are fetched now and used after the rows
                const int pkv = lane < np ? cs[pb + lane].y : 0;
                // moments of candidate c (this lane's view), two candidates ahead
                auto mom_of = [&](int c) -> uint2 {
                    uint2 m = make_uint2(0, 0);
                    if (c < np) {
                        const int pk = __builtin_amdgcn_readlane(pkv, c);
                        if (lane < V) { const MomEntry me = load_mom(mom, (((pk >> 11) & 0x7ff) * sc.W + (pk & 0x7ff)) * V + lane);
                                        m = make_uint2(me.sb, (uint32_t)(((int64_t)mom_db(me) + (int64_t)me.sb * me.sb) / NPX)); }
                    }
                    return m;
                };
                uint2 mb0 = mom_of(0), mb1 = mom_of(1);
                // masked A operands of all region rows (LDS broadcast reads)
                v1l Af[NR];
                {
                    const uint8_t* ra = reg + R * VS + 8 * lh;
#pragma unroll
                    for (int y = 0; y < NR; ++y) {
                        const uint2 w = *(const uint2*)(ra + y * 32);
                        Af[y] = (v1l)((uint64_t)(w.x & bm[0]) | ((uint64_t)(w.y & bm[1]) << 32));
                    }
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const uint8_t* rb = reg + (16 * nt + lx) * VS + 8 * lh;
                    v1l Bf[NR];
#pragma unroll
                    for (int y = 0; y < NR; ++y) {
                        const uint2 w = *(const uint2*)(rb + y * 32);
                        Bf[y] = (v1l)((uint64_t)w.x | ((uint64_t)w.y << 32));
                    }
                    v4i C[RING];
                    int kk = 0;   // next candidate of the pass (sorted by output row)
#pragma unroll
                    for (int y = 0; y < NR; ++y) {
                        const v4i zero = {0, 0, 0, 0};
                        C[y % RING] = __builtin_amdgcn_mfma_i32_16x16x32_i8(
                            Af[y], Bf[y], y == 0 ? zero : C[(y + RING - 1) % RING], 0, 0, 0);
                        if (y >= 2 * WID) {
                            const int j = y - 2 * WID;   // output row
                            while (kk < np) {
                                const int pk = __builtin_amdgcn_readlane(pkv, kk);
                                if (((pk >> 11) & 0x7ff) - yo0 != j) break;
                                const int x = (pk & 0x7ff) - x0;
                                const int xi = x & 3;
                                // S_j at (x, v) = C_{j+2WID} - C_{j-1}; C_{j-1} is slot (y+1) % RING
                                const v4i Cy = C[y % RING];
                                const v4i Cp = j == 0 ? zero : C[(y + 1) % RING];
                                const int val = xi == 0 ? Cy[0] - Cp[0] : xi == 1 ? Cy[1] - Cp[1]
                                              : xi == 2 ? Cy[2] - Cp[2] : Cy[3] - Cp[3];
                                if (lh == (x >> 2)) my_sb[kk * NV + 16 * nt + lx] = val;
                                ++kk;
                            }
                        }
                    }
                }
                STAMP_T(tp1);
                STAMP_ADD(4, tp0, tp1);
                // decision epilogue: one lane per view, as k_score_tiled3
                for (int c = 0; c < np; ++c) {
                    const int k = pb + c;
                    const int ci = __builtin_amdgcn_readfirstlane(cs[k].x);
                    const uint2 mb = mb0;
                    mb0 = mb1;
                    mb1 = mom_of(c + 2);
                    const uint2 ma = make_uint2(__builtin_amdgcn_readlane(mb.x, R),
                                                __builtin_amdgcn_readlane(mb.y, R));
                    const int sab_s = lane < NV ? my_sb[c * NV + lane] : 0;
                    const uint32_t Sab = (uint32_t)(sab_s + 128 * (int)(ma.x + mb.x) - 16384 * NPX);
                    const int32_t da = (int32_t)(__umul24(NPX, ma.y) - __umul24(ma.x, ma.x));
                    const int32_t db = (int32_t)(__umul24(NPX, mb.y) - __umul24(mb.x, mb.x));
                    const int32_t num = (int32_t)(__umul24(NPX, Sab) - __umul24(ma.x, mb.x));
                    const bool live = lane < V && lane != R && da > 0 && db > 0;
                    bool pass = false, guard = false;
                    double ncc = 0.0;
                    if (live) {
                        if (a.thr >= 0.01) {
                            const double L = (double)num * (double)NPX;
                            if (L > 0.0) {
                                const double tk = a.thr * (double)(NPX - 1);
                                const double rhs = (tk * tk) * ((double)da * (double)db);
                                const double diff = L * L - rhs;
                                guard = fabs(diff) <= 1e-8 * rhs;
                                pass = diff > 0.0;
                                if (pass && a.avg) {
                                    const double D = (double)da * (double)db;
                                    double yv = __builtin_amdgcn_rsq(D);
                                    yv = yv * (1.5 - 0.5 * D * yv * yv);
                                    yv = yv * (1.5 - 0.5 * D * yv * yv);
                                    ncc = L * yv * (1.0 / (double)(NPX - 1));
                                }
                            }
                        } else {
                            ncc = ((double)num * (double)NPX) /
                                  ((double)(NPX - 1) * sqrt((double)da * (double)db));
                            guard = fabs(ncc - a.thr) <= kGuard;
                            pass = ncc > a.thr;
                        }
                    }
                    if (__ballot(guard) != 0 && lane == 0)
                        t.fix_list[atomicAdd(t.fix_count, 1)] = ci;
                    const uint64_t m = __ballot(pass);
                    const int cnt = __popcll(m);
                    double avgv = 0.0;
                    if (a.avg && cnt) avgv = wave_sum_dpp(pass ? ncc : 0.0) * c_recip.r[cnt];
                    if (lane == 0) {
                        o_mask[k] = m;
                        o_avg[k] = avgv;
                        o_cnt[k] = cnt;
                    }
                }
                [[maybe_unused]] const int pe = pb + np;
                STAMP_T(tp2);
                STAMP_ADD(5, tp1, tp2);
                STAMP_ADD(6, 0, (unsigned long long)(pe - pb));
            }
        }
        __syncthreads();
        STAMP(2);
        if (tid < nc) {
            const int i = cs[tid].x;
            a.mask[i] = o_mask[tid];
            a.count[i] = o_cnt[tid];
            if (a.avg) a.avg[i] = o_avg[tid];
        }
        __syncthreads();
        STAMP(3);
    }
}

// Re-scores the candidates k_score_tiled3 flagged (a view decision inside the
// guard band) with the direct scorer, whose guard lanes take the numpy-order
// ctNcc; overwrites their mask/count/avg.  One wave per flagged candidate.
// k_score_fix grid: a batch flags a handful of candidates (often none), and
// the kernel (512 registers per lane, scratch) costs ~28 us per launch over
// 256 blocks even when its list is empty; 16 blocks = 64 waves in flight.
// Variant 13 restores the 256-block grid (A/B).
constexpr int kFixBlocks = 16, kFixBlocksWide = 256;

template <int WID, int NS = 1>
__global__ __launch_bounds__(256) void k_score_fix(const SceneDev sc, const ScoreArgs a,
                                                   const TiledArgs t) {
    const int nfix = *t.fix_count;
    for (int k = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); k < nfix;
         k += gridDim.x * 4) {
        const int64_t cand = __builtin_amdgcn_readfirstlane(t.fix_list[k]);
        const int pk = __builtin_amdgcn_readfirstlane(t.cand_pk[cand]);
        const int q = pk & 0x7ff, r = (pk >> 11) & 0x7ff, R = (pk >> 22) & 0x3ff;
        const int words = (sc.V + 63) >> 6;
        wave_score<WID, NS>(sc, R, q, r, a.thr, a.mask + cand * words, a.count + cand,
                            a.avg ? a.avg + cand : nullptr, a.exact_hits);
    }
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
        wave_score_empty<NS>(rec.mask + out * words, rec.count + out, nullptr, words);
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

// Records ev0 on construction and ev1 on destruction (when given): brackets
// exactly one kernel launch on stream s.
struct TimedLaunch {
    hipStream_t s;
    hipEvent_t e1;
    TimedLaunch(hipStream_t s_, hipEvent_t e0, hipEvent_t e1_) : s(s_), e1(e1_) {
        if (e0) (void)hipEventRecord(e0, s);
    }
    ~TimedLaunch() {
        if (e1) (void)hipEventRecord(e1, s);
    }
};

template <int WID>
int launch_score_w(const SceneDev* sc, const ScoreArgs* a, hipStream_t s, hipEvent_t ev0,
                   hipEvent_t ev1) {
    const int64_t blocks = (a->n + 3) / 4;
    if (blocks == 0) return 0;
    TimedLaunch tl(s, ev0, ev1);
    if (sc->V <= 64)
        hipLaunchKernelGGL((k_score<WID, 1>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, *a);
    else if (sc->V <= 128)
        hipLaunchKernelGGL((k_score<WID, 2>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, *a);
    else
        hipLaunchKernelGGL((k_score<WID, 4>), dim3((unsigned)blocks), dim3(256), 0, s, *sc, *a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int WID, int NT>
void launch_mfma(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, hipStream_t s) {
    constexpr size_t lds = MfmaGeom<WID, NT>::BYTES;
    k_score_mfma<WID, NT><<<dim3(kTiledBlocks / 2), dim3(kMThreads), lds, s>>>(*sc, *a, *t);
}

template <int WID, int NT>
void launch_mfma2(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, hipStream_t s) {
    constexpr size_t lds = Mfma2Geom<WID, NT>::BYTES;
    k_score_mfma2<WID, NT><<<dim3(kTiledBlocks), dim3(kM2Threads), lds, s>>>(*sc, *a, *t);
}

template <int WID>
int launch_score_tiled_w(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, int variant,
                         hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    using G = TileGeom<WID>;
    if (a->n == 0) return 0;
    // tile counters, the work-queue head (tile_count[ntiles]) and fix_count:
    // left at zero by the previous batch's k_tile_scan unless zero_first
    if (t->zero_first &&
        hipMemsetAsync(t->tile_count, 0, sizeof(int32_t) * (t->ntiles + 2), s) != hipSuccess)
        return -1;
    launch_bin(sc, a, t, WID, s);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, *t);
    const int nb = (int)std::min<int64_t>((a->n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(256), 0, s, *a, *t);
    const size_t lds = (size_t)G::ROWS * G::NQ * 64 * 4;
    if (variant == 9) {
        if (sc->mom[WID] == nullptr || (sc->V & 3) != 0 || t->chunk > kM2Threads || t->th != kTH ||
            t->tw != kTW)
            return -3;
        {
            TimedLaunch tl(s, ev0, ev1);
            switch ((sc->V + 15) / 16) {
                case 1: launch_mfma2<WID, 1>(sc, a, t, s); break;
                case 2: launch_mfma2<WID, 2>(sc, a, t, s); break;
                case 3: launch_mfma2<WID, 3>(sc, a, t, s); break;
                default: launch_mfma2<WID, 4>(sc, a, t, s); break;
            }
        }
        hipLaunchKernelGGL(k_score_fix<WID>, dim3(variant == 13 ? kFixBlocksWide : kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (variant == 6) {
        if (sc->mom[WID] == nullptr || (sc->V & 3) != 0 || t->chunk > kMChunk || t->th != kMTH ||
            t->tw != kMTW)
            return -3;
        {
            TimedLaunch tl(s, ev0, ev1);
            switch ((sc->V + 15) / 16) {
                case 1: launch_mfma<WID, 1>(sc, a, t, s); break;
                case 2: launch_mfma<WID, 2>(sc, a, t, s); break;
                case 3: launch_mfma<WID, 3>(sc, a, t, s); break;
                default: launch_mfma<WID, 4>(sc, a, t, s); break;
            }
        }
        hipLaunchKernelGGL(k_score_fix<WID>, dim3(variant == 13 ? kFixBlocksWide : kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (variant == 11) {
        // k_score_tiled4 (experimental): 39 % fewer LDS cycles than
        // k_score_tiled3, same time -- the scorer is not LDS-bound
        if (sc->mom[WID] == nullptr || sc->V > 64 || (sc->V & 3) != 0 || t->chunk > kChunk ||
            t->items == nullptr || t->th != kTH || t->tw != kTW)
            return -3;
        const size_t outs = (size_t)t->chunk * (8 + 8 + 4 + 4);
        {
            TimedLaunch tl(s, ev0, ev1);
            if (sc->V == 48) {
                const size_t lds4 = (size_t)2 * G::ROWS * PairGeom<WID>::NP * 2 * 48 * 4 + outs;
                hipLaunchKernelGGL((k_score_tiled4<WID, 48>), dim3(kTiledBlocks), dim3(kT4Threads), lds4, s, *sc, *a, *t);
            } else {
                const size_t lds4 = (size_t)2 * G::ROWS * PairGeom<WID>::NP * 2 * 64 * 4 + outs;
                hipLaunchKernelGGL((k_score_tiled4<WID, 64>), dim3(kTiledBlocks), dim3(kT4Threads), lds4, s, *sc, *a, *t);
            }
        }
        hipLaunchKernelGGL(k_score_fix<WID>, dim3(variant == 13 ? kFixBlocksWide : kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    // default for every window size: k_score_tiled5 at 8 waves/SIMD (64
    // VGPRs; wid 5 0.417 vs 0.426 ms for tiled3, profiles/r01/ab_tiled5_pin_w5.log;
    // wid 4 0.339 vs 0.373 ms despite 4 spilled VGPRs, ab_tiled5_pin_w4.log)
    if (variant == 0 && sc->mom[WID] != nullptr && sc->V <= 64 && (sc->V & 3) == 0 &&
        t->chunk <= kChunk && t->items != nullptr)
        variant = 15;
    if (variant == 14 || variant == 15) {
        if (sc->mom[WID] == nullptr || (sc->V & 3) != 0 || sc->V > 64 || t->chunk > kChunk || t->items == nullptr)
            return -3;
        const size_t outs = (size_t)t->chunk * (8 + 8 + 4 + 4);
        {
            TimedLaunch tl(s, ev0, ev1);
            if (sc->V == 48) {
                const size_t lds3 = (size_t)G::ROWS * G::NQ * 48 * 4 + outs;
                if (variant == 14) hipLaunchKernelGGL((k_score_tiled5<WID, 48, 6>), dim3(kTiledBlocks), dim3(kT5Threads), lds3, s, *sc, *a, *t);
                else hipLaunchKernelGGL((k_score_tiled5<WID, 48, 8>), dim3(kTiledBlocks), dim3(kT5Threads), lds3, s, *sc, *a, *t);
            } else {
                const size_t lds3 = (size_t)G::ROWS * G::NQ * 64 * 4 + outs;
                if (variant == 14) hipLaunchKernelGGL((k_score_tiled5<WID, 64, 6>), dim3(kTiledBlocks), dim3(kT5Threads), lds3, s, *sc, *a, *t);
                else hipLaunchKernelGGL((k_score_tiled5<WID, 64, 8>), dim3(kTiledBlocks), dim3(kT5Threads), lds3, s, *sc, *a, *t);
            }
        }
        hipLaunchKernelGGL(k_score_fix<WID>, dim3(kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (variant == 4 || variant == 5 || variant == 10 || variant == 13 || (variant == 0 && sc->mom[WID] != nullptr)) {
        if (sc->mom[WID] == nullptr || (sc->V & 3) != 0 || t->chunk > kChunk || t->items == nullptr) return -3;
        const size_t outs = (size_t)t->chunk * (8 + 8 + 4 + 4);
        const bool smem = variant == 4;
        {
        TimedLaunch tl(s, ev0, ev1);
        if (sc->V == 48 && variant != 5) {
            const size_t lds3 = (size_t)G::ROWS * G::NQ * 48 * 4 + outs;
            if (smem) hipLaunchKernelGGL((k_score_tiled3<WID, 48, 1>), dim3(kTiledBlocks), dim3(kT3Threads), lds3, s, *sc, *a, *t);
            else hipLaunchKernelGGL((k_score_tiled3<WID, 48, 0>), dim3(kTiledBlocks), dim3(kT3Threads), lds3, s, *sc, *a, *t);
        } else {
            const size_t lds3 = (size_t)G::ROWS * G::NQ * 64 * 4 + outs;
            if (smem) hipLaunchKernelGGL((k_score_tiled3<WID, 64, 1>), dim3(kTiledBlocks), dim3(kT3Threads), lds3, s, *sc, *a, *t);
            else hipLaunchKernelGGL((k_score_tiled3<WID, 64, 0>), dim3(kTiledBlocks), dim3(kT3Threads), lds3, s, *sc, *a, *t);
        }
        }
        hipLaunchKernelGGL(k_score_fix<WID>, dim3(variant == 13 ? kFixBlocksWide : kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    TimedLaunch tl(s, ev0, ev1);
    switch (variant) {
        case 0: hipLaunchKernelGGL((k_score_tiled<WID, 2, 0>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
        case 1: hipLaunchKernelGGL((k_score_tiled<WID, 2, 1>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
        case 2: hipLaunchKernelGGL((k_score_tiled<WID, 0, 0>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
        default: hipLaunchKernelGGL((k_score_tiled<WID, 1, 0>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// V > 64: bin/scan/scatter as for k_score_tiled3, then the view-group scorer,
// the partials' reduction and the guard-band re-score (direct path, NS slots).
template <int WID>
int launch_score_tiledg_w(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, hipStream_t s,
                          hipEvent_t ev0, hipEvent_t ev1) {
    using G = TileGeom<WID>;
    if (a->n == 0) return 0;
    if (sc->mom[WID] == nullptr || (sc->V & 3) != 0 || sc->V > 256 || t->chunk > kChunk ||
        t->groups != (sc->V + 63) / 64 || t->part_cnt == nullptr || t->part_sum == nullptr ||
        t->tw != kTW || t->th != kTH)
        return -3;
    if (t->xq == nullptr || t->items == nullptr) return -3;
    if (t->zero_first &&
        (hipMemsetAsync(t->tile_count, 0, sizeof(int32_t) * (t->ntiles + 2), s) != hipSuccess ||
         hipMemsetAsync(t->xq, 0, sizeof(int32_t) * 8, s) != hipSuccess))
        return -1;
    launch_bin(sc, a, t, WID, s);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, *t);
    const int nb = (int)std::min<int64_t>((a->n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(256), 0, s, *a, *t);
    static_assert(kTiledBlocks % 8 == 0, "queue labels need a multiple of 8 blocks");
    const size_t lds = (size_t)G::ROWS * G::NQ * 64 * 4 + (size_t)t->chunk * (8 + 8 + 4 + 4) +
                       (size_t)kTGWaves * (2 * WID + 1) * 4 * 4;
    {
        TimedLaunch tl(s, ev0, ev1);
        hipLaunchKernelGGL((k_score_tiledg<WID>), dim3(kTiledBlocks), dim3(kTGThreads), lds, s, *sc, *a, *t);
    }
    hipLaunchKernelGGL(k_group_finalize, dim3(nb), dim3(256), 0, s, *a, *t, (2 * WID + 1) * (2 * WID + 1));
    if (sc->V <= 128)
        hipLaunchKernelGGL((k_score_fix<WID, 2>), dim3(kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
    else
        hipLaunchKernelGGL((k_score_fix<WID, 4>), dim3(kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
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

extern "C" int mvs_read_stamps(unsigned long long* out) {
#ifdef MVS_STAMPS
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 4096 * 8) != hipSuccess) return -1;
    return 0;
#else
    (void)out;
    return -3;
#endif
}

extern "C" int mvs_launch_build_gv(const uint8_t* d_stack, uint8_t* d_gv, int V, int H, int W, int Wq,
                                   int Wp, hipStream_t s) {
    hipLaunchKernelGGL(k_build_gv, dim3(4096), dim3(256), 0, s, d_stack, d_gv, V, H, W, Wq, Wp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_build_moments(const SceneDev* sc, int wid, MomEntry* d_mom, hipStream_t s) {
    switch (wid) {
        case 1: hipLaunchKernelGGL(k_moments<1>, dim3(8192), dim3(256), 0, s, *sc, d_mom); break;
        case 2: hipLaunchKernelGGL(k_moments<2>, dim3(8192), dim3(256), 0, s, *sc, d_mom); break;
        case 3: hipLaunchKernelGGL(k_moments<3>, dim3(8192), dim3(256), 0, s, *sc, d_mom); break;
        case 4: hipLaunchKernelGGL(k_moments<4>, dim3(8192), dim3(256), 0, s, *sc, d_mom); break;
        case 5: hipLaunchKernelGGL(k_moments<5>, dim3(8192), dim3(256), 0, s, *sc, d_mom); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_score(const SceneDev* sc, const ScoreArgs* a, int wid, hipStream_t s,
                                hipEvent_t ev0, hipEvent_t ev1) {
    switch (wid) {
        case 1: return launch_score_w<1>(sc, a, s, ev0, ev1);
        case 2: return launch_score_w<2>(sc, a, s, ev0, ev1);
        case 3: return launch_score_w<3>(sc, a, s, ev0, ev1);
        case 4: return launch_score_w<4>(sc, a, s, ev0, ev1);
        case 5: return launch_score_w<5>(sc, a, s, ev0, ev1);
        default: return -2;
    }
}

extern "C" void mvs_tiled_geometry(int W, int H, int mfma, int* tw, int* th, int* ntx, int* nty) {
    *tw = mfma ? kMTW : kTW;
    *th = mfma ? kMTH : kTH;
    *ntx = (W + *tw - 1) / *tw;
    *nty = (H + *th - 1) / *th;
}

extern "C" int mvs_launch_score_tiled(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t,
                                      int wid, int variant, hipStream_t s, hipEvent_t ev0,
                                      hipEvent_t ev1) {
    if (sc->V > 64) {
        switch (wid) {
            case 1: return launch_score_tiledg_w<1>(sc, a, t, s, ev0, ev1);
            case 2: return launch_score_tiledg_w<2>(sc, a, t, s, ev0, ev1);
            case 3: return launch_score_tiledg_w<3>(sc, a, t, s, ev0, ev1);
            case 4: return launch_score_tiledg_w<4>(sc, a, t, s, ev0, ev1);
            case 5: return launch_score_tiledg_w<5>(sc, a, t, s, ev0, ev1);
            default: return -2;
        }
    }
    switch (wid) {
        case 1: return launch_score_tiled_w<1>(sc, a, t, variant, s, ev0, ev1);
        case 2: return launch_score_tiled_w<2>(sc, a, t, variant, s, ev0, ev1);
        case 3: return launch_score_tiled_w<3>(sc, a, t, variant, s, ev0, ev1);
        case 4: return launch_score_tiled_w<4>(sc, a, t, variant, s, ev0, ev1);
        case 5: return launch_score_tiled_w<5>(sc, a, t, variant, s, ev0, ev1);
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

namespace {
__global__ void k_pack_records(RecordsDev rec, int words, int64_t first, int64_t n, int64_t* out) {
    const int w = 8 + words + 3;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = first + k;
        int64_t* o = out + k * w;
        for (int q = 0; q < 3; ++q) o[q] = __double_as_longlong(rec.c[3 * r + q]);
        for (int q = 0; q < 3; ++q) o[3 + q] = __double_as_longlong(rec.n[3 * r + q]);
        o[6] = __double_as_longlong(rec.xy[2 * r]);
        o[7] = __double_as_longlong(rec.xy[2 * r + 1]);
        for (int q = 0; q < words; ++q) o[8 + q] = (int64_t)rec.mask[r * words + q];
        o[8 + words] = (int64_t)(uint32_t)rec.R[r] | ((int64_t)(uint32_t)rec.count[r] << 32);
        o[9 + words] = (int64_t)(uint32_t)rec.cell[2 * r] | ((int64_t)(uint32_t)rec.cell[2 * r + 1] << 32);
        const uint32_t rgba = *(const uint32_t*)(rec.color + 4 * r);
        o[10 + words] = (int64_t)rgba | ((int64_t)rec.accept[r] << 32);
    }
}

__global__ void k_unpack_records(RecordsDev rec, int words, int64_t first, int64_t n, const int64_t* in) {
    const int w = 8 + words + 3;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = first + k;
        const int64_t* o = in + k * w;
        for (int q = 0; q < 3; ++q) rec.c[3 * r + q] = __longlong_as_double(o[q]);
        for (int q = 0; q < 3; ++q) rec.n[3 * r + q] = __longlong_as_double(o[3 + q]);
        rec.xy[2 * r] = __longlong_as_double(o[6]);
        rec.xy[2 * r + 1] = __longlong_as_double(o[7]);
        for (int q = 0; q < words; ++q) rec.mask[r * words + q] = (uint64_t)o[8 + q];
        rec.R[r] = (int32_t)(uint32_t)o[8 + words];
        rec.count[r] = (int32_t)(uint32_t)((uint64_t)o[8 + words] >> 32);
        rec.cell[2 * r] = (int32_t)(uint32_t)o[9 + words];
        rec.cell[2 * r + 1] = (int32_t)(uint32_t)((uint64_t)o[9 + words] >> 32);
        *(uint32_t*)(rec.color + 4 * r) = (uint32_t)o[10 + words];
        rec.accept[r] = (uint8_t)((uint64_t)o[10 + words] >> 32);
    }
}
}  // namespace

extern "C" int mvs_launch_pack_records(RecordsDev rec, int words, int64_t first, int64_t n,
                                       int64_t* out, hipStream_t s) {
    if (n <= 0) return 0;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_records, dim3(blocks), dim3(256), 0, s, rec, words, first, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_unpack_records(RecordsDev rec, int words, int64_t first, int64_t n,
                                         const int64_t* in, hipStream_t s) {
    if (n <= 0) return 0;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_unpack_records, dim3(blocks), dim3(256), 0, s, rec, words, first, n, in);
    return hipGetLastError() == hipSuccess ? 0 : -1;
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

// ===========================================================================
// SfM front-end: Harris keypoints and NCC descriptor matching (the producer of
// the MVS stage's seed tracks; HarrisFeatures.py, SFM.py)
// ===========================================================================
namespace {

DEV int refl101(int i, int n) {     // BORDER_REFLECT_101 for overruns of <= n - 1
    return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

DEV float gv_px(const SceneDev& sc, int v, int y, int x) {
    return (float)sc.gv[((int64_t)v * sc.H + y) * sc.Wp + x];
}

// Sobel(ksize 3, scale 1/8) at (y, x): the scale is folded into the smoothing
// taps, so every product and sum is exact in float32 (integer gray)
DEV void sobel_at(const SceneDev& sc, int v, int y, int x, float& gx, float& gy) {
    gx = 0.f;
    gy = 0.f;
    const int xm = refl101(x - 1, sc.W), xp = refl101(x + 1, sc.W);
    const int ym = refl101(y - 1, sc.H), yp = refl101(y + 1, sc.H);
#pragma unroll
    for (int u = -1; u <= 1; ++u) {
        const float sm = u == 0 ? 0.25f : 0.125f;
        const int yy = refl101(y + u, sc.H);
        gx += sm * (gv_px(sc, v, yy, xp) - gv_px(sc, v, yy, xm));
    }
#pragma unroll
    for (int u = -1; u <= 1; ++u) {
        const float sm = u == 0 ? 0.25f : 0.125f;
        const int xx = refl101(x + u, sc.W);
        gy += sm * (gv_px(sc, v, yp, xx) - gv_px(sc, v, ym, xx));
    }
}

// cv2.cornerHarris(np.float32(gray), 2, 3, k) (HarrisFeatures.py:141; OpenCV
// 4.x cornerEigenValsVecs + calcHarris, scalar path): cov = (dx^2, dx dy,
// dy^2), 2x2 unnormalised box over rows y-1..y and cols x-1..x (both borders
// BORDER_REFLECT_101), R = (float)((double)(a c - b b) - k (a + c)^2)
__global__ void k_harris(const SceneDev sc, int v, double k, float* __restrict__ resp) {
    const int64_t npx = (int64_t)sc.H * sc.W;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npx;
         p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / sc.W), x = (int)(p - (int64_t)y * sc.W);
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int u = -1; u <= 0; ++u)
#pragma unroll
            for (int w = -1; w <= 0; ++w) {
                float gx, gy;
                sobel_at(sc, v, refl101(y + u, sc.H), refl101(x + w, sc.W), gx, gy);
                s0 += gx * gx;
                s1 += gx * gy;
                s2 += gy * gy;
            }
        const float acbb = s0 * s2 - s1 * s1;
        const double t = (double)(s0 + s2);
        resp[p] = (float)((double)acbb - k * t * t);
    }
}

// float -> uint32 key with the same order (for atomicMax)
DEV uint32_t fkey(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
DEV float fkey_inv(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// cv2.dilate(dst, None): 3x3 max, the constant border never wins; the image
// maximum (dst.max() of the dilated map) through one atomic per block
__global__ void k_dilate_max(const float* __restrict__ resp, int H, int W, float* __restrict__ dil,
                             uint32_t* maxkey) {
    __shared__ uint32_t wmax[16];
    uint32_t best = 0;
    const int64_t npx = (int64_t)H * W;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npx;
         p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        float m = -INFINITY;
        for (int u = -1; u <= 1; ++u)
            for (int w = -1; w <= 1; ++w) {
                const int yy = y + u, xx = x + w;
                if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
                m = fmaxf(m, resp[(int64_t)yy * W + xx]);
            }
        dil[p] = m;
        best = max(best, fkey(m));
    }
    for (int off = 32; off > 0; off >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, off, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t b = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) b = max(b, wmax[w]);
        atomicMax(maxkey, b);
    }
}

// dst > 0.01 * dst.max() with NEP-50 float32 arithmetic; one block per row
// counts, a second pass writes [col, row] in np.where's row-major order
template <bool WRITE>
__global__ void k_harris_rows(const float* __restrict__ dil, int H, int W, const uint32_t* maxkey,
                              int32_t* rowcnt, const int32_t* rowoff, int32_t* out, int64_t cap) {
    __shared__ int32_t wcnt[4];
    __shared__ int32_t base;
    const int y = blockIdx.x;
    const float thr = 0.01f * fkey_inv(*maxkey);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) base = WRITE ? rowoff[y] : 0;
    __syncthreads();
    for (int x0 = 0; x0 < W; x0 += 256) {
        const int x = x0 + (int)threadIdx.x;
        const bool f = x < W && dil[(int64_t)y * W + x] > thr;
        const uint64_t m = __ballot(f);
        if (lane == 0) wcnt[wave] = __popcll(m);
        __syncthreads();
        int before = 0;
        for (int w = 0; w < wave; ++w) before += wcnt[w];
        const int total = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (WRITE && f) {
            const int64_t idx = base + before + __popcll(m & ((1ull << lane) - 1ull));
            if (idx < cap) {
                out[2 * idx] = x;
                out[2 * idx + 1] = y;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) base += total;
        __syncthreads();
    }
    if (!WRITE && threadIdx.x == 0) rowcnt[y] = base;
}

__global__ void k_exclusive_scan(const int32_t* in, int n, int32_t* out) {
    __shared__ int32_t part[1024];
    const int tid = threadIdx.x, per = (n + 1023) / 1024;
    const int b = tid * per, e = min(b + per, n);
    int32_t s = 0;
    for (int k = b; k < e; ++k) s += in[k];
    part[tid] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int32_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int32_t r = tid ? part[tid - 1] : 0;
    for (int k = b; k < e; ++k) {
        out[k] = r;
        r += in[k];
    }
    if (tid == 1023) out[n] = part[1023];
}

// getDescFeatures (HarrisFeatures.py:116-133) for in-bounds [row, col]
// points: the flattened (2w+1)^2 window as kDescWords dwords (zero padded)
// plus its exact moments S = sum g, SS = sum g^2
constexpr int kDescWords = 32;
__global__ void k_gather_desc(const SceneDev sc, int v, const int32_t* __restrict__ rc, int64_t n,
                              int wid, uint32_t* __restrict__ desc, int32_t* __restrict__ S,
                              int32_t* __restrict__ SS) {
    // one lane per (point, descriptor dword): 32 lanes per point, the moments
    // reduced across those lanes
    const int nb = 2 * wid + 1, npx = nb * nb;
    const int64_t total = n * kDescWords;
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < ((total + 63) & ~(int64_t)63);
         id += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = id / kDescWords;
        const int k = (int)(id % kDescWords);
        uint32_t wd = 0;
        int32_t s = 0, ss = 0;
        if (i < n) {
            const int r = rc[2 * i], q = rc[2 * i + 1];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int p = 4 * k + b;
                if (p < npx) {
                    const uint32_t g = sc.gv[((int64_t)v * sc.H + r - wid + p / nb) * sc.Wp + q - wid + p % nb];
                    wd |= g << (8 * b);
                    s += (int32_t)g;
                    ss += (int32_t)(g * g);
                }
            }
            desc[id] = wd;
        }
#pragma unroll
        for (int off = kDescWords / 2; off > 0; off >>= 1) {
            s += __shfl_xor(s, off, kDescWords);
            ss += __shfl_xor(ss, off, kDescWords);
        }
        if (i < n && k == 0) {
            S[i] = s;
            SS[i] = ss;
        }
    }
}

DEV uint32_t desc_byte(const uint32_t* d, int p) { return (d[p >> 2] >> (8 * (p & 3))) & 0xffu; }

// Match(desc1, desc2, thr) (HarrisFeatures.py:15-37), one direction: one wave
// per row i, lanes over j.  ncc from the exact integer moments (closed form);
// a value within kGuard of thr is decided by the numpy-order ctNcc; best =
// max ncc > thr with ties to the smallest j; candidates within 1e-12 of the
// best are re-ranked on their numpy-order values.  -1: no ncc above thr.
__global__ __launch_bounds__(256) void k_match_rows(
        const uint32_t* __restrict__ dA, const int32_t* __restrict__ SA, const int32_t* __restrict__ SSA,
        int64_t nA, const uint32_t* __restrict__ dB, const int32_t* __restrict__ SB,
        const int32_t* __restrict__ SSB, int64_t nB, int npx, double thr, int32_t* __restrict__ best) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (i >= nA) return;
    const __attribute__((address_space(4))) uint32_t* di =
        (const __attribute__((address_space(4))) uint32_t*)(dA + i * kDescWords);
    const int64_t si = SA[i], ssi = SSA[i];
    const int64_t da = (int64_t)npx * ssi - si * si;
    double v1 = -2.0, v2 = -2.0;
    int64_t j1 = -1, j2 = -1;
    auto exact = [&](int64_t j) {
        const uint32_t* a = dA + i * kDescWords;
        const uint32_t* b = dB + j * kDescWords;
        return exact_ncc_generic([&](int p) -> int { return (int)desc_byte(a, p); },
                                 [&](int p) -> int { return (int)desc_byte(b, p); }, npx);
    };
    if (da > 0) {
        for (int64_t j = lane; j < nB; j += 64) {
            const uint4* pb = (const uint4*)(dB + j * kDescWords);
            uint32_t sab = 0;
#pragma unroll
            for (int k4 = 0; k4 < kDescWords / 4; ++k4) {
                const uint4 w = pb[k4];
                sab = __builtin_amdgcn_udot4(di[4 * k4], w.x, sab, false);
                sab = __builtin_amdgcn_udot4(di[4 * k4 + 1], w.y, sab, false);
                sab = __builtin_amdgcn_udot4(di[4 * k4 + 2], w.z, sab, false);
                sab = __builtin_amdgcn_udot4(di[4 * k4 + 3], w.w, sab, false);
            }
            const int64_t sj = SB[j], ssj = SSB[j];
            const int64_t db = (int64_t)npx * ssj - sj * sj;
            if (db <= 0) continue;                         // constant window: ncc is NaN
            const int64_t num = (int64_t)npx * (int64_t)sab - si * sj;
            double ncc = (double)(npx * num) / ((double)(npx - 1) * sqrt((double)da * (double)db));
            if (fabs(ncc - thr) <= kGuard) ncc = exact(j);
            if (!(ncc > thr)) continue;
            if (ncc > v1) {
                v2 = v1; j2 = j1;
                v1 = ncc; j1 = j;
            } else if (ncc > v2) {
                v2 = ncc; j2 = j;
            }
        }
    }
    // wave argmax: larger value, then smaller j
    double bv = v1;
    int64_t bj = j1;
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off, 64);
        const int64_t oj = __shfl_xor(bj, off, 64);
        if (ov > bv || (ov == bv && oj >= 0 && (bj < 0 || oj < bj))) { bv = ov; bj = oj; }
    }
    if (bj >= 0) {
        // near ties: re-rank every lane's top two within 1e-12 of the best on
        // their numpy-order ctNcc
        const bool c1 = j1 >= 0 && fabs(v1 - bv) <= 1e-12, c2 = j2 >= 0 && fabs(v2 - bv) <= 1e-12;
        if (__popcll(__ballot(c1)) + __popcll(__ballot(c2)) > 1) {
            double ev = -2.0;
            int64_t ej = -1;
            if (c1) { ev = exact(j1); ej = j1; }
            if (c2) {
                const double e2 = exact(j2);
                if (e2 > ev || (e2 == ev && j2 < ej)) { ev = e2; ej = j2; }
            }
            for (int off = 32; off > 0; off >>= 1) {
                const double ov = __shfl_xor(ev, off, 64);
                const int64_t oj = __shfl_xor(ej, off, 64);
                if (ov > ev || (ov == ev && oj >= 0 && (ej < 0 || oj < ej))) { ev = ov; ej = oj; }
            }
            bj = ej;
        }
    }
    if (lane == 0) best[i] = (int32_t)bj;
}

}  // namespace

extern "C" int mvs_launch_harris(const SceneDev* sc, int v, double k, float* resp, float* dil,
                                 uint32_t* maxkey, int32_t* rowcnt, int32_t* rowoff, hipStream_t s) {
    const int64_t npx = (int64_t)sc->H * sc->W;
    const int blocks = (int)std::min<int64_t>((npx + 255) / 256, 4096);
    if (hipMemsetAsync(maxkey, 0, sizeof(uint32_t), s) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_harris, dim3(blocks), dim3(256), 0, s, *sc, v, k, resp);
    hipLaunchKernelGGL(k_dilate_max, dim3(blocks), dim3(256), 0, s, resp, sc->H, sc->W, dil, maxkey);
    hipLaunchKernelGGL((k_harris_rows<false>), dim3(sc->H), dim3(256), 0, s, dil, sc->H, sc->W, maxkey,
                       rowcnt, nullptr, nullptr, (int64_t)0);
    hipLaunchKernelGGL(k_exclusive_scan, dim3(1), dim3(1024), 0, s, rowcnt, sc->H, rowoff);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_harris_write(const SceneDev* sc, const float* dil, const uint32_t* maxkey,
                                       const int32_t* rowoff, int32_t* out, int64_t cap, hipStream_t s) {
    hipLaunchKernelGGL((k_harris_rows<true>), dim3(sc->H), dim3(256), 0, s, dil, sc->H, sc->W, maxkey,
                       nullptr, rowoff, out, cap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_gather_desc(const SceneDev* sc, int v, const int32_t* rc, int64_t n, int wid,
                                      uint32_t* desc, int32_t* S, int32_t* SS, hipStream_t s) {
    if (n == 0) return 0;
    if (wid < 1 || (2 * wid + 1) * (2 * wid + 1) > 4 * kDescWords) return -2;
    const int blocks = (int)std::min<int64_t>((n * kDescWords + 255) / 256, 4096);
    hipLaunchKernelGGL(k_gather_desc, dim3(blocks), dim3(256), 0, s, *sc, v, rc, n, wid, desc, S, SS);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_match_rows(const uint32_t* dA, const int32_t* SA, const int32_t* SSA, int64_t nA,
                                     const uint32_t* dB, const int32_t* SB, const int32_t* SSB, int64_t nB,
                                     int npx, double thr, int32_t* best, hipStream_t s) {
    if (nA == 0) return 0;
    hipLaunchKernelGGL(k_match_rows, dim3((unsigned)((nA + 3) / 4)), dim3(256), 0, s, dA, SA, SSA, nA, dB,
                       SB, SSB, nB, npx, thr, best);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

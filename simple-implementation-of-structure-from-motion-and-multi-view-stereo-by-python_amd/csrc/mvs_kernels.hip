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
__device__ __forceinline__ double exact_ncc_stack(const SceneDev sc, int R, int v, int q, int r) {
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
//   EPI 0: decision from the binary64 closed form (guard 1e-9 -> numpy order)
//   EPI 1: decision from a binary32 closed form (|err| < 4e-7; guard 1e-5 ->
//          binary64 -> guard 1e-9 -> numpy order); binary64 only for lanes in
//          the guard and, when avg is wanted, for passing lanes
//   REF 0: reference-view words broadcast with v_readlane
//   REF 1: reference-view words re-read by every lane (same LDS address = broadcast)
template <int WID, int NS, bool UNROLL = false, int EPI = 0, int REF = 0, class Fetch,
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
        if constexpr (EPI == 0) {
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
        if (lane == 0) mask_out[s] = m;
        cnt += __popcll(m);
        acc += pass ? ncc : 0.0;
    }
    if (EPI == 1 && !avg_out) {
        if (lane == 0) *count_out = cnt;
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
        wave_score_empty<NS>(a.mask + cand * words, a.count + cand, a.avg ? a.avg + cand : nullptr);
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
constexpr int kBinBlock = 1024, kBinPer = 8;

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
        const int tile = (r / kTH) * t.ntx + (q / kTW);
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

// Exclusive scans of tile counts and work items (one workgroup).
__global__ __launch_bounds__(1024) void k_tile_scan(const TiledArgs t) {
    __shared__ int32_t part_c[1024], part_i[1024];
    const int tid = threadIdx.x;
    const int per = (t.ntiles + 1023) / 1024;
    const int b = tid * per, e = min(b + per, t.ntiles);
    int32_t sc = 0, si = 0;
    for (int k = b; k < e; ++k) {
        const int c = t.tile_count[k];
        sc += c;
        si += (c + t.chunk - 1) / t.chunk;
    }
    part_c[tid] = sc;
    part_i[tid] = si;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        int32_t vc = tid >= off ? part_c[tid - off] : 0;
        int32_t vi = tid >= off ? part_i[tid - off] : 0;
        __syncthreads();
        part_c[tid] += vc;
        part_i[tid] += vi;
        __syncthreads();
    }
    int32_t rc = tid ? part_c[tid - 1] : 0, ri = tid ? part_i[tid - 1] : 0;
    for (int k = b; k < e; ++k) {
        t.tile_off[k] = rc;
        t.item_off[k] = ri;
        const int c = t.tile_count[k];
        rc += c;
        ri += (c + t.chunk - 1) / t.chunk;
    }
    if (tid == 1023) {
        t.tile_off[t.ntiles] = part_c[1023];
        t.item_off[t.ntiles] = part_i[1023];
    }
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
        // stage: wave w copies (row, quad) pairs w, w+4, ...; lane = view
        for (int pq = wave; pq < G::ROWS * G::NQ; pq += 4) {
            const int ry = pq / G::NQ, kq = pq - ry * G::NQ;
            const int y = y0 + ry, gq = kq0 + kq;
            uint32_t val = 0;
            if (lane < V && y >= 0 && y < sc.H && gq >= 0 && gq < sc.Wq)
                val = *(const uint32_t*)(sc.stack + (int64_t)y * sc.row_bytes + (int64_t)gq * V * 4 + lane * 4);
            lds[pq * QS + lane] = val;
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
int launch_score_tiled_w(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, int variant,
                         hipStream_t s) {
    using G = TileGeom<WID>;
    if (a->n == 0) return 0;
    if (hipMemsetAsync(t->tile_count, 0, sizeof(int32_t) * (t->ntiles + 1), s) != hipSuccess) return -1;
    const int64_t per_block = (int64_t)kBinBlock * kBinPer;
    const int nbin = (int)((a->n + per_block - 1) / per_block);
    hipLaunchKernelGGL(k_bin, dim3(nbin), dim3(kBinBlock), (size_t)t->ntiles * 4, s, *sc, *a, *t, WID);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, *t);
    const int nb = (int)std::min<int64_t>((a->n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(256), 0, s, *a, *t);
    const size_t lds = (size_t)G::ROWS * G::NQ * 64 * 4;
    switch (variant) {
        case 0: hipLaunchKernelGGL((k_score_tiled<WID, 0, 0>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
        case 1: hipLaunchKernelGGL((k_score_tiled<WID, 1, 0>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
        case 2: hipLaunchKernelGGL((k_score_tiled<WID, 0, 1>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
        default: hipLaunchKernelGGL((k_score_tiled<WID, 1, 1>), dim3(kTiledBlocks), dim3(256), lds, s, *sc, *a, *t); break;
    }
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

extern "C" void mvs_tiled_geometry(int W, int H, int* ntx, int* nty) {
    *ntx = (W + kTW - 1) / kTW;
    *nty = (H + kTH - 1) / kTH;
}

extern "C" int mvs_launch_score_tiled(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t,
                                      int wid, int variant, hipStream_t s) {
    if (sc->V > 64) return -3;
    switch (wid) {
        case 1: return launch_score_tiled_w<1>(sc, a, t, variant, s);
        case 2: return launch_score_tiled_w<2>(sc, a, t, variant, s);
        case 3: return launch_score_tiled_w<3>(sc, a, t, variant, s);
        case 4: return launch_score_tiled_w<4>(sc, a, t, variant, s);
        case 5: return launch_score_tiled_w<5>(sc, a, t, variant, s);
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

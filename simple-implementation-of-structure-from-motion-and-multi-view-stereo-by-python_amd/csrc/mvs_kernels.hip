// HIP kernels for the MVS2 photo-consistency hot path (gfx950 / CDNA4).
//
// Reference path (MarvinChung/simple-implementation-of-structure-from-motion-
// and-multi-view-stereo-by-python):
//   MyPatch.photo_consistenecy_test   MVS2.py:62-77   -> k_score_mma / k_score
//   projectPoint                      utils.py:241-244 -> project()
//   getDescFeatures                   HarrisFeatures.py:116-133 -> window gather
//   ctNcc                             MVS2.py:39-43   -> integer moments + exact_ncc_*
//   patch_expansion candidate geometry + accept test MVS2.py:329-369 -> k_expand*
//
// Numerics.  Window sums are exact integers (S_a, S_aa, S_b, S_bb, S_ab) and
// the NCC is n (n S_ab - S_a S_b) / ((n-1) sqrt((n S_aa - S_a^2)(n S_bb - S_b^2))).
// Every decision close to the threshold is taken again on the numpy-order
// ctNcc (exact_ncc_*), so every accept/reject is the reference's.  Geometry is
// binary64 in the reference's order; this file is compiled with
// -ffp-contract=off (products that numpy/OpenBLAS fuse are written as fma()).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <utility>

#include <hipcub/hipcub.hpp>

#include "mvs_device.h"
#include "mvs_mma.h"

namespace {

// ctNcc of view R's and view v's windows at (q, r) in numpy's operation order
// (the guard-band path: rare).  Both windows' rows come in with every load in
// flight at once (one memory round trip), aligned to the window's first
// column (alignbyte) and held as packed bytes; the numpy-order arithmetic
// then reads every pixel from a register (constant indices: fully unrolled).
// Reading pixel by pixel from memory in the serial loops cost ~20 us per call
// (one dependent load per pixel and pass): a single such pair in a sweep set
// the whole k_score_fix launch (26 us at wid 3, profiles/r06/).
template <int WID>
__device__ __noinline__ double exact_ncc_stack(const SceneDev sc, int R, int v, int q, int r) {
    constexpr int NB = 2 * WID + 1, NPX = NB * NB;
    constexpr int NW = (NB + 3) / 4, ND = NW + 1;   // aligned dwords per row, dwords loaded per row
    const int64_t vstride = (int64_t)sc.V * 4;
    const int o = (q - WID) & 3;
    const uint8_t* p0 = sc.stack + (int64_t)(r - WID) * sc.row_bytes + (int64_t)((q - WID) >> 2) * vstride;
    // one window's rows, every load in flight, aligned to column q - WID
    auto window = [&](int view, uint32_t (&w)[NB][NW]) {
        uint32_t d[NB][ND];
#pragma unroll
        for (int row = 0; row < NB; ++row)
#pragma unroll
            for (int j = 0; j < ND; ++j)
                d[row][j] = *(const uint32_t*)(p0 + (int64_t)row * sc.row_bytes + j * vstride + view * 4);
#pragma unroll
        for (int row = 0; row < NB; ++row)
#pragma unroll
            for (int j = 0; j < NW; ++j) w[row][j] = __builtin_amdgcn_alignbyte(d[row][j + 1], d[row][j], o);
    };
    uint32_t wa[NB][NW], wb[NB][NW];
    window(R, wa);
    __builtin_amdgcn_sched_barrier(0);   // the second window's loads after: fewer registers in flight
    window(v, wb);
    // pixel i as a double, re-extracted at every use (opaque): kept as packed
    // bytes, not as NPX live doubles per window
    auto px = [&](const uint32_t (&w)[NB][NW], int i) -> double {
        const uint32_t word = (uint32_t)opaque((int)w[i / NB][(i % NB) >> 2]);
        return (double)((word >> (8 * ((i % NB) & 3))) & 255u);
    };
    int sa = 0, sb = 0;
#pragma unroll
    for (int i = 0; i < NPX; ++i) {
        sa += (int)((wa[i / NB][(i % NB) >> 2] >> (8 * ((i % NB) & 3))) & 255u);
        sb += (int)((wb[i / NB][(i % NB) >> 2] >> (8 * ((i % NB) & 3))) & 255u);
    }
    const double ma = (double)sa / NPX, mb = (double)sb / NPX;
    // numpy's pairwise sum of (x - mean)^2 for 8 <= n <= 128: 8 accumulators,
    // combined pairwise, the remainder added in order (as pairwise_sq)
    static_assert(NPX >= 8 && NPX <= 128, "numpy pairwise summation restated for 8 <= n <= 128");
    auto pw = [&](const uint32_t (&w)[NB][NW], double m) -> double {
        double acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { const double x = px(w, j) - m; acc[j] = x * x; }
#pragma unroll
        for (int i = 8; i < NPX - (NPX % 8); i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) { const double x = px(w, i + j) - m; acc[j] += x * x; }
        double res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
#pragma unroll
        for (int i = NPX - (NPX % 8); i < NPX; ++i) { const double x = px(w, i) - m; res += x * x; }
        return res;
    };
    const double stda = sqrt(pw(wa, ma) / NPX), stdb = sqrt(pw(wb, mb) / NPX);
    // sum(d1 * d2) with Python's sequential sum (MVS2.py:43)
    double acc = 0;
#pragma unroll
    for (int i = 0; i < NPX; ++i) acc = acc + ((px(wa, i) - ma) / stda) * ((px(wb, i) - mb) / stdb);
    return acc / (NPX - 1);
}

DEV int wave_reduce_add(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

DEV double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// ---------------------------------------------------------------------------
// Direct photo test: one wave per candidate, lane l handles views l, l+64, ...
// (NS slots); window rows gathered from the stack.  Used for small batches,
// for the guard-band re-score of the tiled scorer (k_score_fix) and for the
// children of small expansion sweeps.
// ---------------------------------------------------------------------------
// One wave scores one candidate whose window sits at (q, r) of every view
// (the reference samples all views at view R's pixel, MVS2.py:68).
// fetch(s, row, j) returns the j-th dword (4 pixels of this lane's view of
// slot s) of window row `row`, counted from the quad holding column q - WID;
// o = (q - WID) & 3.  Lane 0 of the wave writes mask/count/avg.
// Decision without sqrt/div: for thr >= 0.01, ncc > thr  <=>  L > 0 and
// L^2 > thr^2 (n-1)^2 da db  with L = n*num (exact in binary64); a relative band
// of 1e-11 around it (5e-12 relative on the NCC) goes to the numpy-order
// path.  The comparison itself is exact to ~6e-16 relative (L is an exact
// integer, rhs three roundings); the reference's numpy-order NCC differs from
// the exact value by < 1e-14 relative (121 terms, std from pairwise sums), so
// the band covers every pair whose reference decision could differ from the
// exact one with a margin of ~500.  (It was 1e-8: 104 numpy-order
// evaluations per wid-3 sweep then, most of k_score_fix's 26 us.)
template <int WID, int NS, class Fetch>
DEV void wave_score_core(const SceneDev& sc, int R, int q, int r, double thr, Fetch&& fetch,
                         uint64_t* mask_out, int32_t* count_out, double* avg_out, int32_t* exact_hits) {
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
    // one view slot: every row's loads in flight at once (a latency-bound
    // wave per candidate); more slots: one row at a time (registers)
    constexpr int ROW_UNROLL = NS == 1 ? NB : 1;
#pragma unroll ROW_UNROLL
    for (int row = 0; row < NB; ++row) {
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
        if (live) {
            if (thr >= 0.01) {
                const double L = (double)((int64_t)NPX * num);
                if (L > 0.0) {
                    const double tk = thr * (double)(NPX - 1);
                    const double rhs = (tk * tk) * ((double)da * (double)db);
                    const double diff = L * L - rhs;
                    if (fabs(diff) <= 1e-11 * rhs) {
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
                ncc = (double)((int64_t)NPX * num) / ((double)(NPX - 1) * sqrt((double)da * (double)db));
                if (fabs(ncc - thr) <= kGuard) {
                    ncc = exact_ncc_stack<WID>(sc, R, v, q, r);
                    atomicAdd(exact_hits, 1);
                }
                pass = ncc > thr;
            }
        }
        const uint64_t m = __ballot(pass);
        // NS slots can exceed the candidate's ceil(V/64) mask words (NS = 4 for
        // 128 < V <= 192): only the words that exist are written
        if (lane == 0 && 64 * s < V) mask_out[s] = m;
        cnt += __popcll(m);
        acc += pass ? ncc : 0.0;
    }
    if (!avg_out || cnt == 0) {
        if (lane == 0) {
            if (count_out) *count_out = cnt;
            if (avg_out) *avg_out = 0.0;
        }
        return;
    }
    const double tot = wave_sum(acc);
    if (lane == 0) {
        if (count_out) *count_out = cnt;
        *avg_out = tot / cnt;
    }
}

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
    wave_score_core<WID, NS>(sc, R, q, r, thr, fetch, mask_out, count_out, avg_out, exact_hits);
}

template <int NS>
DEV void wave_score_empty(uint64_t* mask_out, int32_t* count_out, double* avg_out, int words) {
    const int lane = threadIdx.x & 63;
    if (lane < NS && lane < words) mask_out[lane] = 0;
    if (lane == 0) {
        if (count_out) *count_out = 0;
        if (avg_out) *avg_out = 0.0;
    }
}

// ---------------------------------------------------------------------------
// Scene setup: RGB (V, H, W, 3) -> gray (OpenCV BGR2GRAY fixed point applied to
// the RGB data, HarrisFeatures.py:125 on main.py:18's RGB images), written in
// both layouts.  A block takes one image row, a 64-pixel strip and 16 views at
// a time: the RGB bytes come in as whole 16-byte pieces, gv rows leave as 64-B
// runs per view and stack quads as 64-B runs per quad (16 views).
// ---------------------------------------------------------------------------
constexpr int kSceneStrip = 64, kSceneViews = 16;

__global__ __launch_bounds__(256) void k_build_scene(const SceneDev sc, const uint8_t* __restrict__ rgb,
                                                     uint8_t* __restrict__ stack, uint8_t* __restrict__ gv) {
    __shared__ __attribute__((aligned(16))) uint8_t srgb[kSceneViews][kSceneStrip * 3];
    __shared__ uint32_t squad[kSceneStrip / 4][kSceneViews];
    const int y = blockIdx.y;
    const int x0 = blockIdx.x * kSceneStrip;
    const int nx = min(kSceneStrip, sc.W - x0);
    const int tid = threadIdx.x;
    const bool vec = (sc.W & 15) == 0;          // every strip is whole 16-byte pieces
    for (int v0 = 0; v0 < sc.V; v0 += kSceneViews) {
        const int nv = min(kSceneViews, sc.V - v0);
        if (vec) {
            const int cpv = nx * 3 / 16;
            for (int k = tid; k < nv * cpv; k += 256) {
                const int vv = k / cpv, c = k - vv * cpv;
                *(uint4*)(&srgb[vv][16 * c]) =
                    *(const uint4*)(rgb + (((int64_t)(v0 + vv) * sc.H + y) * sc.W + x0) * 3 + 16 * c);
            }
        } else {
            for (int k = tid; k < nv * nx * 3; k += 256) {
                const int vv = k / (nx * 3), b = k - vv * (nx * 3);
                srgb[vv][b] = rgb[(((int64_t)(v0 + vv) * sc.H + y) * sc.W + x0) * 3 + b];
            }
        }
        __syncthreads();
        {
            const int vv = tid >> 4, qd = tid & 15;
            if (vv < nv && 4 * qd < nx) {
                uint32_t word = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int x = 4 * qd + b;
                    if (x < nx) {
                        const uint8_t* p = &srgb[vv][3 * x];
                        const uint32_t g = (p[0] * 1868u + p[1] * 9617u + p[2] * 4899u + 8192u) >> 14;
                        word |= g << (8 * b);
                    }
                }
                squad[qd][vv] = word;
                // gv: signed bytes s = g - 128 (the tiled scorer's operands)
                *(uint32_t*)(gv + ((int64_t)(v0 + vv) * sc.H + y) * sc.Wp + x0 + 4 * qd) = word ^ 0x80808080u;
            }
        }
        __syncthreads();
        {
            const int qd = tid >> 4, vv = tid & 15;
            if (vv < nv && 4 * qd < nx)
                *(uint32_t*)(stack + (int64_t)y * sc.row_bytes + ((int64_t)(x0 / 4 + qd) * sc.V + v0 + vv) * 4) =
                    squad[qd][vv];
        }
        __syncthreads();
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
        wave_score_empty<NS>(a.mask + cand * a.mstride, a.count ? a.count + cand : nullptr,
                             a.avg ? a.avg + cand * a.astride : nullptr, words);
        return;
    }
    q = __builtin_amdgcn_readfirstlane(q);
    r = __builtin_amdgcn_readfirstlane(r);
    wave_score<WID, NS>(sc, R, q, r, a.thr, a.mask + cand * a.mstride, a.count ? a.count + cand : nullptr,
                        a.avg ? a.avg + cand * a.astride : nullptr, a.exact_hits);
}

// ---------------------------------------------------------------------------
// Tiled scorer, stage 1: candidates binned by the 16x8 pixel tile of their
// window centre.  k_bin projects (binary64, reference order), tests the
// window and ranks the candidate inside its tile -- through an LDS histogram
// per block (one global atomic per non-empty (block, tile) pair) when the tile
// counters fit in LDS, else through one global atomic per candidate -- and
// writes it into the tile's bucket.  k_item_scan then writes the work items
// (tile, chunk j: candidates [j chunk, (j+1) chunk) of its bucket) in tile
// order; the scorers read the tile's final count when they take the item
// (item_desc).
// ---------------------------------------------------------------------------
// MVS_BIN_PER (mvs_internal.h): candidates per k_bin thread (A/B switch)
#ifdef MVS_STAMPS
// diagnostic build only: per-workgroup cycle sums of the scorer's phases
// (slot 0 items, 1 staging + barrier, 2 moments, 3 candidates, 4 wave 0's own
// candidate time, 5 wave 0's M-blocks), read by mvs_read_stamps; k_bin's
// workgroups use rows 2048 + (slot 0 workgroups, 1 projection + LDS ranks,
// 2 global tile bases, 3 bucket writes)
__device__ unsigned long long g_stamps[4096 * 16];
#define STAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(slot, val) \
    do { if (threadIdx.x == 0) atomicAdd(&g_stamps[(blockIdx.x & 4095) * 16 + (slot)], (unsigned long long)(val)); } while (0)
#define STAMP_ADD_W0(slot, val) \
    do { if ((threadIdx.x & 1023) == 0) atomicAdd(&g_stamps[(blockIdx.x & 4095) * 16 + (slot)], (unsigned long long)(val)); } while (0)
// any lane / one lane per wave
#define STAMP_ADD_ANY(slot, val) atomicAdd(&g_stamps[(blockIdx.x & 4095) * 16 + (slot)], (unsigned long long)(val))
#define STAMP_ADD_LANE0(slot, val) \
    do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_stamps[(blockIdx.x & 4095) * 16 + (slot)], (unsigned long long)(val)); } while (0)
#define STAMP_ADD_ROW(row, slot, val) \
    do { if (threadIdx.x == 0) atomicAdd(&g_stamps[((row) & 4095) * 16 + (slot)], (unsigned long long)(val)); } while (0)
#else
#define STAMP_ADD_ROW(row, slot, val)
#define STAMP(var)
#define STAMP_ADD(slot, val)
#define STAMP_ADD_W0(slot, val)
#define STAMP_ADD_ANY(slot, val)
#define STAMP_ADD_LANE0(slot, val)
#endif

constexpr int kBinBlock = MVS_BIN_BLOCK, kBinPer = MVS_BIN_PER, kBinLdsTiles = 16384;
static_assert(kBinBlock * kBinPer == MVS_BIN_CHUNK, "MVS_BIN_CHUNK candidates per k_bin workgroup");
static_assert(kBinBlock * kBinPer <= 4096, "k_bin_count packs a rank inside the workgroup into 12 bits");
#ifndef MVS_IMPLICIT_MEAN
#define MVS_IMPLICIT_MEAN 64   // A/B switch (a huge value keeps k_item_scan everywhere)
#endif
constexpr int64_t kImplicitMean = MVS_IMPLICIT_MEAN;
constexpr int kMmaGrid = 256;         // the scorers' workgroups: one per CU; the queue balances

// The work items in tile order: one workgroup reads every tile's count, scans
// the tiles' chunk counts (chunk j of a tile: bucket entries [j chunk,
// (j+1) chunk) below min(count, cap)) and writes (tile, j) for each chunk into
// segment 0 (the other segments' counts to 0).  Measured against items in the
// order k_bin's workgroups opened them (same box): k_score_mma_v at ring256
// 1.67-1.72 vs 1.86-1.87 ms per 2^20, k_score_tab at dinoRing 105.5-107.2 vs
// 111.1-111.6 us (profiles/r04/r4r_*, r4s_*).
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_item_scan(const TiledArgs t) {
    __shared__ int s_w[kScanThreads / 64 + 1];
    const int per = (t.ntiles + kScanThreads - 1) / kScanThreads;   // tiles per thread, contiguous
    const int t0 = min((int)threadIdx.x * per, t.ntiles), t1 = min(t0 + per, t.ntiles);
    int mine = 0;
    for (int k = t0; k < t1; ++k) {
        const int c = min(t.tile_count[k * kTcStride], t.cap);
        mine += (c + t.chunk - 1) / t.chunk;
    }
    int incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d, 64);
        if ((threadIdx.x & 63) >= d) incl += o;
    }
    if ((threadIdx.x & 63) == 63) s_w[threadIdx.x >> 6] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) { const int c = s_w[w]; s_w[w] = run; run += c; }
        s_w[kScanThreads / 64] = run;
    }
    __syncthreads();
    int slot = s_w[threadIdx.x >> 6] + incl - mine;
    for (int k = t0; k < t1; ++k) {
        const int c = min(t.tile_count[k * kTcStride], t.cap);
        for (int j = 0; j * t.chunk < c; ++j) t.items[slot++] = make_int4(k, j, 0, 0);
    }
    if (threadIdx.x < kItemSegs) t.n_items[32 * threadIdx.x] = threadIdx.x == 0 ? s_w[kScanThreads / 64] : 0;
}

template <bool LDSHIST>
__global__ __launch_bounds__(kBinBlock) void k_bin(const SceneDev sc, const ScoreArgs a,
                                                   const TiledArgs t, int wid, const MomentsDev mt) {
    extern __shared__ int32_t hist[];      // [ntiles] local counts, then global bases
    // the cameras' projection constants (R', t, fx fy cx cy) in LDS: every
    // candidate reads its reference camera's 16 values there instead of by
    // per-lane global loads.  Field-major ([value][view]): the lanes of a
    // read (one value of 64 random views) fall in distinct banks; view-major
    // rows of 128 B put them all in two banks (81 % of k_bin's LDS cycles
    // were bank conflicts, profiles/r06/pmc_r6e_w5_scorer.csv)
    __shared__ double s_cam[16][MVS_MAX_VIEWS];
    const int words = (sc.V + 63) >> 6;
    const int64_t base = (int64_t)blockIdx.x * kBinBlock * kBinPer;
    // every candidate's inputs in flight at once (one memory round trip, not
    // one per candidate), issued before the camera table's loads: the two
    // round trips overlap (k_bin 27.4 vs 28.5 us, profiles/r06/r6k_*)
    int Rk[kBinPer];
    double ck[kBinPer][3];
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
        const int64_t i = base + (int64_t)k * kBinBlock + threadIdx.x;
        const int64_t ii = i < a.n ? i : 0;
        Rk[k] = a.ref[ii];
        ck[k][0] = a.c[3 * ii];
        ck[k][1] = a.c[3 * ii + 1];
        ck[k][2] = a.c[3 * ii + 2];
    }
    for (int k = threadIdx.x; k < sc.V * 16; k += blockDim.x) {
        const int v = k >> 4, f = k & 15;
        const CamDev& cm = sc.cams[v];
        s_cam[f][v] = f < 9 ? cm.Rp[f] : f < 12 ? cm.t[f - 9] : f == 12 ? cm.fx : f == 13 ? cm.fy : f == 14 ? cm.cx : cm.cy;
    }
    STAMP(t0);
    // the previous batch's counter set (the other parity; its k_score_fix
    // has finished, stream order) back to zero for the batch after this one
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < t.zero_words; k += (int64_t)gridDim.x * blockDim.x)
        t.zero_blk[k] = 0;
    if (LDSHIST)
        for (int b = threadIdx.x; b < t.ntiles; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    int tl[kBinPer], lr[kBinPer], pk[kBinPer];
    // a candidate whose reference window is constant (D_a = 0: ctNcc's std is
    // 0, every view's NCC nan, MVS2.py:41-42) passes no view: its outputs are
    // written here (V = [], avg 0) and it is not binned, so the scorers never
    // see it.  Decided from the scene's constant-window bits (MomentsDev.flat,
    // 2 B per pixel and 16 views: an L2 hit), one gather per candidate, all of
    // a thread's in flight
    const uint16_t* __restrict__ flat = mt.flat;
    int fk[kBinPer];
    int qk[kBinPer], rk[kBinPer];
    // V = [], avg 0.  Records (a.rec, V <= 64): one 16-B store.  No loop
    // with a run-time trip count here: the compiler's wait-count tracking
    // then stays exact, where a loop made it wait for every store of the
    // thread (vmcnt(0)) before the first (workgroup, tile) atomic
    auto settle = [&](int64_t i) {
        if (a.rec && words == 1) {
            *(uint4*)(a.mask + 2 * i) = make_uint4(0u, 0u, 0u, 0u);
            return;
        }
#pragma unroll
        for (int w = 0; w < MVS_MAX_VIEWS / 64; ++w)
            if (w < words) a.mask[i * a.mstride + w] = 0;
        if (a.count) a.count[i] = 0;
        if (a.avg) a.avg[i * a.astride] = 0.0;
    };
    // Every load of these two loops is issued and consumed on every path
    // (past the batch: candidate 0's values; invalid window: pixel (0, 0)'s
    // bits), so that no path leaves a load pending at the loops' joins: the
    // compiler's wait counting then stays exact, where a conditionally
    // consumed load made it wait for every memory operation of the thread
    // (vmcnt(0): the xy and settled stores included) ahead of the barrier
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
        const int64_t i = base + (int64_t)k * kBinBlock + threadIdx.x;
        const int R = Rk[k];
        const double c[3] = {ck[k][0], ck[k][1], ck[k][2]};
        double px, py;
        project_vals([&](int f) { return s_cam[f][R]; }, c, px, py);
        int q = 0, r = 0;
        const bool inb = i < a.n, ok = inb && window_ok(sc, px, py, wid, &q, &r);
        if (!ok) q = r = 0;
        tl[k] = ok ? 0 : inb ? -1 : -2;   // -2: past the batch
        qk[k] = q;
        rk[k] = r;
        // the stores ahead of the bit load: the wait for the last load then
        // waits for nothing behind it
        if (inb) {
            a.xy[2 * i] = px;
            a.xy[2 * i + 1] = py;
        }
        if (inb && !ok) settle(i);
        fk[k] = flat ? flat[((int64_t)r * sc.W + q) * (mt.VP >> 4) + (R >> 4)] : 0;
    }
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
        const bool cst = (fk[k] >> (Rk[k] & 15)) & 1;
        if (tl[k] < 0) continue;
        const int64_t i = base + (int64_t)k * kBinBlock + threadIdx.x;
        if (cst) {
            tl[k] = -1;
            settle(i);
            continue;
        }
        const int R = Rk[k], q = qk[k], r = rk[k];
        const int tx = q / MVS_TILE_W, ty = r / MVS_TILE_H;
        const int tile = ty * t.ntx + tx;
        tl[k] = tile;
        pk[k] = (q - tx * MVS_TILE_W) | ((r - ty * MVS_TILE_H) << 4) | (R << 7);
        if (LDSHIST) {
            lr[k] = atomicAdd(&hist[tile], 1);
        } else {
            lr[k] = atomicAdd(&t.tile_count[tile * kTcStride], 1);
            // implicit items: the candidate that opens chunk j >= 1 appends it
            if (t.implicit && lr[k] > 0 && lr[k] < t.cap && lr[k] % t.chunk == 0)
                t.items[t.item_seg + atomicAdd(&t.n_items[32], 1)] = make_int4(tile, lr[k] / t.chunk, 0, 0);
        }
    }
    STAMP(t1);
    if (LDSHIST) {
        // the workgroup's base in every tile it touched: every thread's
        // returning atomics in flight together (ntiles <= 16 x 1024)
        __syncthreads();
        int bs[kBinLdsTiles / kBinBlock];
#pragma unroll
        for (int j = 0; j < kBinLdsTiles / kBinBlock; ++j) {
            const int b = threadIdx.x + j * kBinBlock;
            const int c = b < t.ntiles ? hist[b] : 0;
            bs[j] = c ? atomicAdd(&t.tile_count[b * kTcStride], c) : 0;
        }
        auto bs_tile = [&](int jj) { return (int)threadIdx.x + jj * kBinBlock; };
        if (t.implicit) {
            // implicit items: the workgroup whose share of a tile's bucket
            // holds the first entry of chunk j >= 1 (below cap) appends (tile, j)
#pragma unroll
            for (int j = 0; j < kBinLdsTiles / kBinBlock; ++j) {
                const int b = bs_tile(j);
                const int c = b < t.ntiles ? hist[b] : 0;
                const int end = min(bs[j] + c, t.cap);
                for (int q = max((bs[j] + t.chunk - 1) / t.chunk, 1); c > 0 && q * t.chunk < end; ++q)
                    t.items[t.item_seg + atomicAdd(&t.n_items[32], 1)] = make_int4(b, q, 0, 0);
            }
        }
        __syncthreads();   // every thread has read the counts it needs
#pragma unroll
        for (int j = 0; j < kBinLdsTiles / kBinBlock; ++j) {
            const int b = bs_tile(j);
            if (b < t.ntiles) hist[b] = bs[j];
        }
        __syncthreads();
    }
    STAMP(t2);
    // straight into the tile's bucket (no separate scatter pass); past the
    // bucket's capacity to the direct path's list (counted: mvs_scorer_stats)
    int over = 0;
#pragma unroll
    for (int k = 0; k < kBinPer; ++k) {
        const int64_t i = base + (int64_t)k * kBinBlock + threadIdx.x;
        if (tl[k] < 0) continue;
        const int rank = (LDSHIST ? hist[tl[k]] : 0) + lr[k];
        if (rank < t.cap) {
            t.sorted[(int64_t)tl[k] * t.cap + rank] = make_int2((int32_t)i, pk[k]);
        } else {
            t.fix_list[atomicAdd(t.fix_count, 1)] = make_int4((int32_t)i, tl[k], pk[k], 0);
            ++over;
        }
    }
    if (t.stats && __ballot(over != 0)) {
        over = wave_reduce_add(over);
        if ((threadIdx.x & 63) == 0) atomicAdd(&t.stats[1], (unsigned long long)over);
    }
    STAMP(t3);
    STAMP_ADD_ROW(2048 + blockIdx.x, 0, 1);
    STAMP_ADD_ROW(2048 + blockIdx.x, 1, t1 - t0);
    STAMP_ADD_ROW(2048 + blockIdx.x, 2, t2 - t1);
    STAMP_ADD_ROW(2048 + blockIdx.x, 3, t3 - t2);
}

// ---------------------------------------------------------------------------
// Tiled scorer, stage 2: the candidates of a 16x8 pixel tile against every
// view on the matrix cores (v_mfma_i32_16x16x64_i8 over the tile's window
// region), one workgroup of 16 waves per CU taking work items from a dynamic
// queue: k_score_mma for V <= 64 (every view staged), k_score_mma_v for V > 64
// (64-view groups).  Both decide each (candidate, view) pair from exact
// integer window products and moments (see k_score_mma).
// ---------------------------------------------------------------------------
constexpr int kMmaThreads = 1024, kMmaWaves = kMmaThreads / 64;
constexpr int kGroupViews = MVS_GROUP_VIEWS;   // views per view group (V > 64): one mask word
constexpr int kMmaChunk = MVS_MMA_CHUNK;       // candidates per work item, V <= 64 (<= 1024: the scorers' lists)
constexpr int kGroupChunk = MVS_GROUP_CHUNK;   // candidates per work item, V > 64 (reference windows staged)
constexpr int kSortBins = MVS_TILE_H / 2;   // k_score_mma sorts an item's candidates by row pair

// ---------------------------------------------------------------------------
// k_score_mma (V <= 64).  A workgroup (16 waves) takes one work item (the
// candidates of one 16x8 pixel tile, at most kMmaChunk) from a dynamic queue:
//   1. the item's window region of every view (signed bytes s = g - 128,
//      [view][ROWS rows][32 columns], two aligned 16-B loads of gv per view
//      row) and its candidate list go to LDS; the NEXT item's region is
//      loaded into registers meanwhile (issued after this item is staged,
//      written to LDS at the top of the next iteration), so the global
//      latency hides behind phases 2-3;
//   2. per (pixel, view) of the tile: S_b and w = 1/sqrt(n S_bb - S_b^2) in
//      binary64 (NaN for a constant window: ctNcc's nan, never passes), from
//      horizontal v_dot4_i32_i8 prefix sums and vertical sums;
//   3. 16 candidates per wave and M-block: C[m][v] = sum over the window of
//      s_R s_v by v_mfma_i32_16x16x64_i8 (A = the reference window masked to
//      candidate m's window, B = view v's region), exact;
//   4. per (candidate, view): num = n C - S_a S_b (the n S_ab - S_a S_b of
//      ctNcc, shift invariant), ncc = n/(n-1) num w_a w_b, so
//      ncc > thr  <=>  num w_b > T = thr (n-1)/(n w_a): one binary32 fma,
//      with a relative guard band of 2e-6 |T| (the binary32 roundings add
//      < 3e-7 |T|); a candidate with any pair in the band is re-scored by
//      k_score_fix (numpy-order ctNcc).  avg_ncc_score = n/(n-1) w_a
//      sum(num w_b) / cnt in binary64.
// ---------------------------------------------------------------------------
// a candidate's constants in phase 3 (per wave, 32 slots: the two M-blocks
// of its unit)
struct alignas(16) CandInfo {
    int32_t osb;              // LDS byte offset of its pixel's S_b table row (the w row follows from it)
    int32_t Sa;               // -S_a
    int32_t R;                // reference view (-1: no candidate)
    float T;                  // decision threshold on num w_b (FAST: binary32; else thr)
};

// LDS layout: region | S_b table, w table (binary64), [w table (binary32)]
// (the tables alias the horizontal sums of phase 2) | per-wave candidate
// slots | the item's candidates | 32 zero bytes
struct MmaLds {
    int reg, regsz, sb, w, wf, ci, wp, cand, zero, total;
};

// Dynamic LDS of k_score_mma.  DB: the two region buffers and the two
// candidate buffers are static LDS arrays of the kernel (the next item's
// region and candidates land by LDS-DMA during this item's candidates), so
// the dynamic part holds only the tables and slots; otherwise one region and
// one candidate buffer come first.  WF: a binary32 copy of the w table.
template <int WID, int NBLK, bool WF, bool DB>
__host__ __device__ constexpr MmaLds mma_lds(int V) {
    using G = MmaGeom<WID>;
    constexpr int VP = 16 * NBLK;
    MmaLds L{};
    L.reg = 0;
    L.regsz = V * G::VS;                               // VS is a multiple of 32
    L.sb = DB ? 0 : L.regsz;
    L.w = L.sb + 128 * VP * 4;
    L.wf = L.w + 128 * VP * 8;
    const int htmp = G::ROWS * 16 * VP * 4, tab = 128 * VP * (WF ? 16 : 12);
    L.ci = L.sb + (htmp > tab ? htmp : tab);
    L.wp = L.ci + kMmaWaves * 32 * (int)sizeof(CandInfo);
    L.cand = L.wp;
    L.zero = L.cand + (DB ? 0 : kMmaChunk * 8);
    L.total = L.zero + 32;
    return L;
}

// static LDS of k_score_mma: region and candidate buffers (DB) + small slots
template <int WID, int NBLK, bool DB>
__host__ __device__ constexpr int mma_static_lds() {
    return (DB ? 2 * (16 * NBLK * MmaGeom<WID>::VS + 16 + kMmaChunk * 8) : 64) + 8 + 4 + 65 * 8 + 64 +
           kSortBins * kMmaWaves * 3;   // the row sort's counts and offsets
}

// what fits in 160 KiB beside the rest at this NBLK (1 workgroup of 16 waves
// per CU): double buffering first, then the binary32 w copy
template <int WID, int NBLK>
__host__ __device__ constexpr bool mma_db() {
    return mma_lds<WID, NBLK, false, true>(16 * NBLK).total + mma_static_lds<WID, NBLK, true>() <= 160 * 1024;
}
template <int WID, int NBLK>
__host__ __device__ constexpr bool mma_wf() {
    return mma_lds<WID, NBLK, true, mma_db<WID, NBLK>()>(16 * NBLK).total +
               mma_static_lds<WID, NBLK, mma_db<WID, NBLK>()>() <= 160 * 1024;
}
template <int WID, int NBLK>
__host__ __device__ constexpr MmaLds mma_layout(int V) {
    return mma_lds<WID, NBLK, mma_wf<WID, NBLK>(), mma_db<WID, NBLK>()>(V);
}

template <int WID, int NBLK, bool FAST>
__global__ __launch_bounds__(kMmaThreads) void k_score_mma(const SceneDev sc, const ScoreArgs a, const TiledArgs t,
                                                           const int4* __restrict__ items,
                                                           const int2* __restrict__ sorted) {
    using G = MmaGeom<WID>;
    constexpr int NB = G::NB, NPX = G::NPX, ROWS = G::ROWS, KS = G::KS, VS = G::VS, C0 = G::C0;
    constexpr int VP = 16 * NBLK;                         // views per table row
    constexpr bool WF = mma_wf<WID, NBLK>(), DB = mma_db<WID, NBLK>();
    constexpr int RPV = VS / 32;                          // region rows per view incl. the pad row
    constexpr int PF = (VP * RPV * 2 + kMmaThreads - 1) / kMmaThreads;   // 16-B pieces per thread
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // DB: the two region and candidate buffers are distinct LDS objects, so
    // that the compiler sees that reads of one do not alias the LDS-DMA into
    // the other (no vmcnt wait for the prefetch before them)
    // (DB) each region buffer ends in 16 zero bytes, never an LDS-DMA target:
    // phase 3 reads a window row or the zeros by an offset select inside the
    // one buffer, so that the read keeps the buffer's alias scope and does not
    // wait for the other buffer's LDS-DMA (a select between two LDS objects
    // would wait for every LDS-DMA in flight)
    constexpr int RB = DB ? VP * VS : 16, CB = DB ? kMmaChunk * 8 : 16;
    __shared__ __attribute__((aligned(16))) uint8_t s_reg0[RB + 16], s_reg1[RB + 16];
    __shared__ __attribute__((aligned(16))) uint8_t s_cand0[CB], s_cand1[CB];
    __shared__ int s_ids[2];
    __shared__ int s_simd_n[4];
    __shared__ int s_V;
    __shared__ double s_recip[65];
    // the item's candidates are reordered by pixel row inside the tile (a
    // counting sort in LDS): per (wave, row) counts and destination offsets
#ifdef MVS_STAMPS
    __shared__ unsigned s_maxown;
    if (threadIdx.x == 0) s_maxown = 0;
#endif
    __shared__ __attribute__((aligned(16))) uint8_t s_rcnt[kSortBins][kMmaWaves];
    __shared__ __attribute__((aligned(16))) int16_t s_roff[kSortBins][kMmaWaves];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int V = sc.V;
    const int npiece = V * RPV * 2;
    // k / V as umulhi(k, ceil(2^32 / V)): exact for k V < 2^32 (uniform, once)
    const uint32_t vmagic = __builtin_amdgcn_readfirstlane(0xffffffffu / (uint32_t)V + 1u);
    if (tid <= 64) s_recip[tid] = c_recip.r[tid];
    if (tid == 0) s_V = V;
    const MmaLds L = mma_layout<WID, NBLK>(V);
    uint32_t* htmp = (uint32_t*)(smem + L.sb);
    int32_t* tsb = (int32_t*)(smem + L.sb);
    double* tw = (double*)(smem + L.w);
    float* twf = (float*)(smem + L.wf);
    CandInfo* ci = (CandInfo*)(smem + L.ci) + wave * 32;
    if (tid < 8) ((uint32_t*)(smem + L.zero))[tid] = 0u;
    if (DB && tid >= 8 && tid < 16) ((uint32_t*)((tid < 12 ? s_reg0 : s_reg1) + RB))[tid & 3] = 0u;
    const int zoff = DB ? RB : L.zero - L.reg;   // the zero row, relative to a region buffer

    const double kn = (double)NPX / (double)(NPX - 1);
    const float tqf = (float)(a.thr / kn);
    ItemMap im;
    im.load(t);
    const int n_units = im.total();
    int32_t* head = t.head;

    // The region of an item (gv rows, signed bytes) goes to LDS by LDS-DMA
    // (global_load_lds_dwordx4: 64 lanes x 16 B land contiguously), 32 B per
    // region row and RPV rows per view including one pad row, so that the
    // image is linear in the piece index; rows outside the image are clamped
    // (their pixels are never inside a valid window).
    auto region_buf = [&](int buf) -> uint8_t* { return DB ? (buf ? s_reg1 : s_reg0) : smem + L.reg; };
    auto cand_buf = [&](int buf) -> uint8_t* { return DB ? (buf ? s_cand1 : s_cand0) : smem + L.cand; };
    auto stage = [&](const int4 d, auto bufc) {
        constexpr int buf = decltype(bufc)::value;
        const int ty = d.x / t.ntx, tx = d.x - ty * t.ntx;
        const int x0 = tx * MVS_TILE_W, yr0 = ty * MVS_TILE_H - WID;
        uint8_t* base = region_buf(buf);
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int k = tid + p * kMmaThreads;
            if (k < npiece) {
                const int v = k / (2 * RPV), r2 = k - v * (2 * RPV);
                const int y = min(max(yr0 + (r2 >> 1), 0), sc.H - 1);
                const uint8_t* src = sc.gv + ((int64_t)v * sc.H + y) * sc.Wp + (x0 - 8) + 16 * (r2 & 1);
                __builtin_amdgcn_global_load_lds((const void*)src,
                                                 (void __attribute__((address_space(3)))*)(base + (p * kMmaThreads + wave * 64) * 16),
                                                 16, 0, 0);
            }
        }
        // the item's sorted (id, pk) entries, one dword per lane
        uint8_t* cbase = cand_buf(buf);
        const int32_t* csrc = (const int32_t*)(sorted + d.y);
#pragma unroll
        for (int p = 0; p < 2 * kMmaChunk / kMmaThreads; ++p) {
            const int k = tid + p * kMmaThreads;
            if (k < 2 * d.z)
                __builtin_amdgcn_global_load_lds((const void*)(csrc + k),
                                                 (void __attribute__((address_space(3)))*)(cbase + (p * kMmaThreads + wave * 64) * 4),
                                                 4, 0, 0);
        }
    };

    // Work items flow through a pipeline: while item k is scored, item k+1's
    // region (DB) and candidate list, item k+2's descriptor and thread 0's
    // claim of item k+3 are in flight; the barrier that ends item k retires them.
    if (tid == 0) {
        s_ids[0] = atomicAdd(head, 1);
        s_ids[1] = atomicAdd(head, 1);
    }
    // The 16 waves sit 4 to a SIMD, which shares its issue among them: work is
    // split by SIMD (virtual wave vw = 4 SIMD + rank on it) where it does not
    // divide evenly over the waves.  vw = wave unless every SIMD holds 4 waves.
    if (tid < 4) s_simd_n[tid] = 0;
    __syncthreads();
    const int simd = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // HW_ID.SIMD_ID
    int srank = 0;
    if (lane == 0) srank = atomicAdd(&s_simd_n[simd & 3], 1);
    srank = __builtin_amdgcn_readfirstlane(srank);
    __syncthreads();
    const bool simd_ok = s_simd_n[0] == 4 && s_simd_n[1] == 4 && s_simd_n[2] == 4 && s_simd_n[3] == 4;
    const int vw = __builtin_amdgcn_readfirstlane(simd_ok ? 4 * (simd & 3) + srank : wave);
    int cur = __builtin_amdgcn_readfirstlane(s_ids[0]);
    int nx1 = __builtin_amdgcn_readfirstlane(s_ids[1]);
    if (cur >= n_units) return;
    int4 dcur = item_desc(t, items, im, cur);
    dcur = make_int4(__builtin_amdgcn_readfirstlane(dcur.x), __builtin_amdgcn_readfirstlane(dcur.y),
                     __builtin_amdgcn_readfirstlane(dcur.z), 0);
    stage(dcur, std::integral_constant<int, 0>{});
    // item nx1's descriptor (uniform, scalar loads) and thread 0's claim of
    // the item after it
    int4 dnx1 = nx1 < n_units ? item_desc(t, items, im, nx1) : make_int4(0, 0, 0, 0);
    int pend = 0;
    if (tid == 0) pend = atomicAdd(head, 1);
    __syncthreads();   // everyone has read s_ids before they are rewritten

    // one round per work item; the rounds alternate the buffers (DB), with the
    // buffer index a compile-time constant in each
    auto round = [&](auto bufc) -> bool {
        constexpr int buf = decltype(bufc)::value;
        STAMP(t0);
        const int nc = dcur.z;
            const uint8_t* reg = region_buf(buf);
            const int2* cand = (const int2*)cand_buf(buf);
            // ---- 1. this item's region and candidates are staged ----
            if (tid == 0) s_ids[0] = pend;
            __syncthreads();
            const int nx2 = __builtin_amdgcn_readfirstlane(s_ids[0]);
            STAMP(t1);
            // thread -> (row, view) maps of phase 2, from a V read after the
            // barrier (not hoisted: no registers held across phase 3)
            const int Vl = s_V;
            // tasks split into four contiguous SIMD segments (vw = 4 SIMD + rank):
            // each SIMD issues a quarter of them whatever the task count
            const int ploc = (vw & 3) * 64 + lane, pseg = vw >> 2;
            const int hq = (Vl * ROWS + 3) >> 2, vq = (Vl * 16 + 3) >> 2;   // per-SIMD quotas
            const int vtask = pseg * vq + ploc;
            const int h_rho0 = (int)__umulhi((uint32_t)vtask, vmagic), h_v0 = vtask - h_rho0 * Vl;   // vertical: (column, view)
            const bool m2 = ploc < vq && vtask < Vl * 16;
            // sort of the candidates by pixel row pair (rrel >> 1: a K-step's two
            // region rows), stable: thread k holds candidate k; its rank among
            // the wave's candidates of its row pair now, the destination after
            // the offsets are known (phase 2 barriers)
            int2 my_c = make_int2(0, 0);
            int my_row = kSortBins, my_rank = 0;
            if (tid < nc) {
                my_c = ((const int2*)cand_buf(buf))[tid];
                my_row = (my_c.y >> 5) & 3;
            }
            int my_cnt = 0;   // lane y < kSortBins: the wave's count of bin y
            static_for<kSortBins>([&](auto Yc) {
                constexpr int y = Yc;
                const uint64_t bm = __ballot(my_row == y);
                if (my_row == y) my_rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                my_cnt = writelane<y>((uint32_t)my_cnt, (uint32_t)__popcll(bm));
            });
            if (lane < kSortBins) s_rcnt[lane][wave] = (uint8_t)my_cnt;
            // ---- 2. S_b and w of every view at the tile's pixels ----
            // horizontal sums of each region row on the unsigned bytes g = s + 128
            // (the moments are shift invariant): prefix sums by v_sad_u8 and
            // v_dot4_u32_u8, packed as (sum g^2) << 12 | sum g
            for (int j = 0; ploc + 256 * j < hq; ++j) {
                const int k = pseg * hq + ploc + 256 * j;
                if (k < V * ROWS) {
                    const int rho = (int)__umulhi((uint32_t)k, vmagic), v = k - rho * Vl;
                    const uint4 lo = *(const uint4*)(reg + v * VS + rho * 32);
                    const uint4 hi = *(const uint4*)(reg + v * VS + rho * 32 + 16);
                    const uint32_t d[8] = {lo.x ^ 0x80808080u, lo.y ^ 0x80808080u, lo.z ^ 0x80808080u,
                                           lo.w ^ 0x80808080u, hi.x ^ 0x80808080u, hi.y ^ 0x80808080u,
                                           hi.z ^ 0x80808080u, hi.w ^ 0x80808080u};
                    uint32_t PS[33], PQ[33];
                    PS[0] = 0;
                    PQ[0] = 0;
    #pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint32_t m1 = d[k] & 0xffu, m2b = d[k] & 0xffffu, m3 = d[k] & 0xffffffu;
                        PS[4 * k + 1] = __builtin_amdgcn_sad_u8(m1, 0u, PS[4 * k]);
                        PS[4 * k + 2] = __builtin_amdgcn_sad_u8(m2b, 0u, PS[4 * k]);
                        PS[4 * k + 3] = __builtin_amdgcn_sad_u8(m3, 0u, PS[4 * k]);
                        PS[4 * k + 4] = __builtin_amdgcn_sad_u8(d[k], 0u, PS[4 * k]);
                        PQ[4 * k + 1] = __builtin_amdgcn_udot4(m1, d[k], PQ[4 * k], false);
                        PQ[4 * k + 2] = __builtin_amdgcn_udot4(m2b, d[k], PQ[4 * k], false);
                        PQ[4 * k + 3] = __builtin_amdgcn_udot4(m3, d[k], PQ[4 * k], false);
                        PQ[4 * k + 4] = __builtin_amdgcn_udot4(d[k], d[k], PQ[4 * k], false);
                    }
                    uint32_t* hrow = htmp + rho * 16 * VP + v;
    #pragma unroll
                    for (int x = 0; x < 16; ++x)
                        hrow[x * VP] = ((PQ[x + C0 + NB] - PQ[x + C0]) << 12) | (PS[x + C0 + NB] - PS[x + C0]);
                }
            }
            __syncthreads();
            STAMP(t1a);
            // destination offsets of the row sort: row y's candidates start after
            // every candidate of rows < y, then by wave (lane y of the last wave:
            // the row's 16 wave counts in one read, prefix sums in registers)
            if (wave == kMmaWaves - 1 && lane < kSortBins) {
                const uint4 q4 = *(const uint4*)&s_rcnt[lane][0];
                const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
                int pre[kMmaWaves];
                int tot = 0;
    #pragma unroll
                for (int w = 0; w < kMmaWaves; ++w) {
                    pre[w] = tot;
                    tot += (qw[w >> 2] >> (8 * (w & 3))) & 0xff;
                }
                int ex = tot;
    #pragma unroll
                for (int off = 1; off < kSortBins; off <<= 1) {
                    const int yv = __shfl_up(ex, off, 64);
                    if (lane >= off) ex += yv;
                }
                const int base = ex - tot;
                uint32_t pk[kMmaWaves / 2];
    #pragma unroll
                for (int w = 0; w < kMmaWaves / 2; ++w)
                    pk[w] = (uint32_t)(base + pre[2 * w]) | ((uint32_t)(base + pre[2 * w + 1]) << 16);
                *(uint4*)&s_roff[lane][0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                *(uint4*)&s_roff[lane][8] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
            }
            // vertical sums -> (S_b of s, w) per (pixel, view); the table overwrites
            // the horizontal sums, so every thread reads first
            int ms[MVS_TILE_H];
            double mw[MVS_TILE_H];
            const int m2x = h_rho0, m2v = h_v0;   // thread -> (pixel column, view)
            if (m2) {
                int S[ROWS], Q[ROWS];
    #pragma unroll
                for (int rho = 0; rho < ROWS; ++rho) {
                    const uint32_t h = htmp[(rho * 16 + m2x) * VP + m2v];
                    S[rho] = (int)(h & 0xfffu);
                    Q[rho] = (int)(h >> 12);
                }
                int sg = 0, q = 0;
    #pragma unroll
                for (int rho = 0; rho < NB; ++rho) {
                    sg += S[rho];
                    q += Q[rho];
                }
    #pragma unroll
                for (int y = 0; y < MVS_TILE_H; ++y) {
                    if (y > 0) {
                        sg += S[y + NB - 1] - S[y - 1];
                        q += Q[y + NB - 1] - Q[y - 1];
                    }
                    const int db = NPX * q - sg * sg;   // < 2^31: n * sum g^2 <= 121 * 121 * 255^2
                    // v_rsq_f64 + one Newton step: max relative error 4.1e-15 over
                    // 4M values of D < 2^31 (tools/ubench/rsq_acc.hip; 5.2e-8 without).
                    // A constant window (D = 0) gets rsq = inf and then nan from the
                    // Newton step: ctNcc's nan, which never passes (no select)
                    const double D = (double)db;
                    double w = __builtin_amdgcn_rsq(D);
                    w = w * (1.5 - 0.5 * D * w * w);
                    ms[y] = sg - 128 * NPX;             // S_b of s = g - 128
                    mw[y] = w;
                }
            }
            __syncthreads();
            STAMP(t1b);
            if (tid < nc) ((int2*)cand_buf(buf))[s_roff[my_row][wave] + my_rank] = my_c;
            if (m2)
    #pragma unroll
                for (int y = 0; y < MVS_TILE_H; ++y) {
                    const int o = (y * 16 + m2x) * VP + m2v;
                    tsb[o] = ms[y];
                    tw[o] = mw[y];
                    if constexpr (WF) twf[o] = (float)mw[y];
                }
            if (VP > V)   // views V..VP-1 of the last 16-view block: never pass
                for (int k = tid; k < 128 * (VP - V); k += kMmaThreads) {
                    const int px = k / (VP - V), v = V + (k - px * (VP - V));
                    tsb[px * VP + v] = 0;
                    tw[px * VP + v] = __builtin_nan("");
                    if constexpr (WF) twf[px * VP + v] = __builtin_nanf("");
                }
            __syncthreads();
            STAMP(t2);
            // the next items' loads, in flight during phase 3 (phase 2's register
            // spills would otherwise wait for them: vmcnt retires in order): item
            // nx1's region and candidates (DB), item nx2's descriptor (scalar
            // loads) and thread 0's claim of the item after it
            if (nx1 < n_units) {
                if constexpr (DB) stage(dnx1, std::integral_constant<int, buf ^ 1>{});
            }
            int4 dnx2 = make_int4(0, 0, 0, 0);
            if (nx2 < n_units) {
                dnx2 = item_desc(t, items, im, nx2);
                if (tid == 0) pend = atomicAdd(head, 1);
            }
    
            // ---- 3. + 4. the candidates: units of two M-blocks of 16 (32
            // consecutive candidates of the row-sorted list), which share their
            // K-steps and B operands and give the epilogue two independent
            // chains.  The SIMDs share the issue of their waves, so the blocks
            // are split into four contiguous SIMD segments of equal size; a
            // segment's waves take its units (the last one may be a single
            // block) ----
            const int nblk = (nc + 15) >> 4;
            const int sg = vw >> 2, sr = vw & 3;           // SIMD segment, wave rank in it
            const int seg_b = (nblk * sg) >> 2, seg_e = (nblk * (sg + 1)) >> 2;
    #ifdef MVS_STAMPS
            unsigned long long w0blk = 0;
    #endif
            for (int fb = seg_b + 2 * sr; fb < seg_e; fb += 8) {
              const int nh = min(2, seg_e - fb);
    #ifdef MVS_STAMPS
              w0blk += nh;
    #endif
              auto unit = [&](auto nhc) {
                constexpr int NH = decltype(nhc)::value;
                // lane constants recomputed per unit (hoisted, they would hold
                // registers through phase 2)
                const int ol = opaque(lane);
                const int m = ol & 15, kh = ol >> 4;
                int2 e[NH];
                bool valid[NH];
                int qrel[NH], rrel[NH], Rv[NH];
    #pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const int kk = (fb + h) * 16 + m;
                    valid[h] = kk < nc;
                    e[h] = valid[h] ? cand[kk] : make_int2(-1, 0);
                    qrel[h] = e[h].y & 15;
                    rrel[h] = (e[h].y >> 4) & 7;
                    Rv[h] = e[h].y >> 7;
                }
                // the candidates' constants (row 0 of the wave computes them for
                // both blocks, before the K-loop: they do not depend on it), shared
                // through LDS
                double my_wa[NH];
    #pragma unroll
                for (int h = 0; h < NH; ++h) my_wa[h] = 0.0;
                if (kh == 0) {
    #pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        CandInfo c;
                        const int px = e[h].y & 127;          // rrel * 16 + qrel
                        const int o = px * VP + Rv[h];
                        const double wa = tw[o];
                        c.osb = L.sb + px * VP * 4;
                        c.Sa = -tsb[o];                       // -S_a: num = n C + (-S_a) S_b
                        c.R = valid[h] ? Rv[h] : -1;
                        // FAST: T = thr (n-1)/n sqrt(da) in binary32 (1-ulp reciprocal,
                        // well inside the guard band); else the decision is on ncc
                        c.T = FAST ? (valid[h] ? tqf * __builtin_amdgcn_rcpf((float)wa) : __builtin_nanf("")) : 0.0f;
                        ci[16 * h + m] = c;
                        my_wa[h] = wa;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                // the unit's candidates are sorted by row pair: its window rows lie
                // in candidate 0's pair to the last valid candidate's pair + NB - 1
                const int last = min(16 * NH - 1, nc - 1 - fb * 16);
                const int r_lo = __builtin_amdgcn_readlane(rrel[0], 0) & ~1;
                const int r_hi = (last >= 16 ? __builtin_amdgcn_readlane(rrel[NH - 1], last - 16)
                                             : __builtin_amdgcn_readlane(rrel[0], last)) | 1;
                constexpr int KSK = WID + 1;     // K-steps of one row's windows
                const int s_lo = r_lo >> 1, s_hi = (r_hi + NB - 1) >> 1;
                const int span = s_hi - s_lo + 1;
                // A: the reference windows, masked to each candidate's window
                // columns (this lane's 16 columns) and rows (bit 2s: K-step s holds
                // a window row of this lane's row parity)
                uint32_t cm[NH][4], rb[NH];
    #pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const uint32_t wm = valid[h] ? (((1u << NB) - 1u) << (qrel[h] + C0)) : 0u;
                    const uint32_t hm = wm >> (16 * (kh & 1));
    #pragma unroll
                    for (int k4 = 0; k4 < 4; ++k4) cm[h][k4] = byte_mask((hm >> (4 * k4)) & 15u);
                    rb[h] = valid[h] ? (((1u << NB) - 1u) << rrel[h]) >> (kh >> 1) : 0u;
                }
                const int lofs = 32 * (kh >> 1) + 16 * (kh & 1);
                v4i C[NH][NBLK];
    #pragma unroll
                for (int h = 0; h < NH; ++h)
    #pragma unroll
                    for (int nb = 0; nb < NBLK; ++nb) C[h][nb] = (v4i){0, 0, 0, 0};
                // NST K-steps from sb; steps below sd are done (their A rows read zeros)
                // steps [SAFE_LO, SAFE_HI] of the pass hold window rows of every
                // candidate of the unit (no row test there)
                auto kpass = [&](auto nstc, auto safe_lo_c, auto safe_hi_c, int sb, int sd) {
                    constexpr int NST = decltype(nstc)::value;
                    constexpr int SAFE_LO = decltype(safe_lo_c)::value, SAFE_HI = decltype(safe_hi_c)::value;
                    uint32_t rbp[NH];
                    int aoff[NH];
    #pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        rbp[h] = (rb[h] & ~((1u << (2 * sd)) - 1u)) >> (2 * sb);
                        aoff[h] = Rv[h] * VS + lofs + 64 * sb;
                    }
                    const uint8_t* bptr[NBLK];
    #pragma unroll
                    for (int nb = 0; nb < NBLK; ++nb) bptr[nb] = reg + min(16 * nb + m, V - 1) * VS + lofs + 64 * sb;
                    // operands of step st + 1 load while step st's MFMAs run; the
                    // schedule barrier keeps the compiler from hoisting more loads
                    // (their registers would spill)
                    uint4 av[2][NH], bv[2][NBLK];
                    auto load = [&](int st, int slot) {
    #pragma unroll
                        for (int h = 0; h < NH; ++h)
                            // rows outside the window read 16 zero bytes: an offset
                            // select instead of a branch around the load
                            av[slot][h] = *(const uint4*)(reg + ((st >= SAFE_LO && st <= SAFE_HI) ||
                                                                         ((rbp[h] >> (2 * st)) & 1u)
                                                                     ? aoff[h] + 64 * st : zoff));
    #pragma unroll
                        for (int nb = 0; nb < NBLK; ++nb) bv[slot][nb] = *(const uint4*)(bptr[nb] + 64 * st);
                    };
                    load(0, 0);
    #pragma unroll
                    for (int st = 0; st < NST; ++st) {
                        const int cur = st & 1;
                        if (st + 1 < NST) load(st + 1, cur ^ 1);
                        v4i A[NH];
    #pragma unroll
                        for (int h = 0; h < NH; ++h)
                            A[h] = (v4i){(int)(av[cur][h].x & cm[h][0]), (int)(av[cur][h].y & cm[h][1]),
                                         (int)(av[cur][h].z & cm[h][2]), (int)(av[cur][h].w & cm[h][3])};
    #pragma unroll
                        for (int nb = 0; nb < NBLK; ++nb) {
                            const v4i B = {(int)bv[cur][nb].x, (int)bv[cur][nb].y, (int)bv[cur][nb].z, (int)bv[cur][nb].w};
    #pragma unroll
                            for (int h = 0; h < NH; ++h)
                                C[h][nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[h], B, C[h][nb], 0, 0, 0);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
                // one row pair (span KSK, from s_lo <= KS - KSK): steps 1 .. KSK-2
                // hold rows of every window; two (span KSK+1): steps 2 .. KSK-2
                using I = std::integral_constant<int, 0>;
                if (span <= KSK) {
                    kpass(std::integral_constant<int, KSK>{}, std::integral_constant<int, 1>{},
                          std::integral_constant<int, KSK - 2>{}, min(s_lo, KS - KSK), 0);
                } else if (span == KSK + 1) {
                    kpass(std::integral_constant<int, KSK + 1>{}, std::integral_constant<int, 2>{},
                          std::integral_constant<int, KSK - 2>{}, min(s_lo, KS - KSK - 1), 0);
                } else {
                    for (int sd = s_lo; sd <= s_hi; sd += KSK)
                        kpass(std::integral_constant<int, KSK>{}, std::integral_constant<int, KSK>{}, I{},
                              min(sd, KS - KSK), sd);
                }
                // lane (kh, m) holds C[h][nb][i] = block h's candidate 4 kh + i, view 16 nb + m
                uint32_t pmv[NH], gdv[NH];
    #pragma unroll
                for (int h = 0; h < NH; ++h) pmv[h] = gdv[h] = 0u;
                double sacc[NH][4];
                static_for<4>([&](auto Ic) {
                    constexpr int i = Ic;
    #pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const CandInfo c = ci[16 * h + 4 * kh + i];
                        const int32_t* sbp = (const int32_t*)(smem + c.osb) + m;
                        const double* twp = (const double*)(smem + L.w + 2 * (c.osb - L.sb)) + m;
                        const float* twfp = (const float*)(smem + c.osb + (L.wf - L.sb)) + m;   // WF only
                        const float gT = 2e-6f * fabsf(c.T);
                        // slow path: n/(n-1) w_a from the pixel's w row
                        double ca = 0.0;
                        if constexpr (!FAST) ca = kn * twp[(c.R < 0 ? 0 : c.R) - m];
                        double sa = 0.0;
                        uint64_t g = 0;
                        float ax[NBLK];   // FAST: the decision values, for the guard test
                        static_for<NBLK>([&](auto Nc) {
                            constexpr int nb = Nc;
                            const int vl = 16 * nb + m;
                            const int num = __mul24(c.Sa, sbp[16 * nb]) + __mul24(NPX, C[h][nb][i]);
                            const double w = twp[16 * nb];
                            uint64_t P;
                            if constexpr (FAST) {
                                // ncc > thr <=> num w_b > T; a constant window (w_b = 0 here)
                                // never passes.  The candidate's own view R passes (its ncc
                                // is n/(n-1) > thr): its mask bit and its term of the sum
                                // are taken out once per candidate, not tested per pair
                                const float x = fmaf((float)num, WF ? twfp[16 * nb] : (float)w, -c.T);
                                P = __builtin_amdgcn_fcmpf(x, 0.0f, 2);                         // ogt
                                ax[nb] = x;
                                // the sum's term in the passing lanes only
                                sa = fma_f64_lanes(sa, num, w, P);
                            } else {
                                const double ncc = (double)num * w * ca;
                                const bool pass = vl != c.R && ncc > a.thr;
                                P = __ballot(pass);
                                g |= __ballot(vl != c.R && fabs(ncc - a.thr) <= kGuard);
                                sa = fma((double)num, pass ? w : 0.0, sa);
                            }
                            pmv[h] = writelane<2 * (i * NBLK + nb)>(pmv[h], (uint32_t)P);
                            pmv[h] = writelane<2 * (i * NBLK + nb) + 1>(pmv[h], (uint32_t)(P >> 32));
                        });
                        if constexpr (FAST) {
                            // guard band: min over the views of |x| < gT (one compare)
                            float mn = fabsf(ax[0]);
    #pragma unroll
                            for (int nb = 1; nb < NBLK; ++nb) mn = fminf(mn, fabsf(ax[nb]));
                            g = __builtin_amdgcn_fcmpf(mn, gT, 4);                               // olt
                        }
                        gdv[h] = writelane<2 * i>(gdv[h], (uint32_t)g);
                        gdv[h] = writelane<2 * i + 1>(gdv[h], (uint32_t)(g >> 32));
                        sacc[h][i] = sa;
                    }
                });
                // owner lane c = 4 j + i (row 0) of each block's candidate c: its mask
                // bits, guard bits and sum from the lanes that hold them (crossbar
                // permutes, no LDS storage)
                const int jj = m >> 2, ii = m & 3;
    #pragma unroll
                for (int h = 0; h < NH; ++h) {
                    uint64_t mk = 0;
    #pragma unroll
                    for (int nb = 0; nb < NBLK; ++nb) {
                        const uint32_t d = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (2 * (ii * NBLK + nb) + (jj >> 1)), (int)pmv[h]);
                        mk |= (uint64_t)((d >> (16 * (jj & 1))) & 0xffffu) << (16 * nb);
                    }
                    const uint32_t gw = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (2 * ii + (jj >> 1)), (int)gdv[h]);
                    const bool gg = ((gw >> (16 * (jj & 1))) & 0xffffu) != 0u;
                    double mine = 0.0;
                    if (a.avg != nullptr) {
                        const double rs = row_sum16_x4(sacc[h], m);
                        const int src = 4 * (16 * jj + ii);   // lane 16 j + i holds candidate 4 j + i's sum
                        const unsigned long long rb64 = __double_as_longlong(rs);
                        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)rb64);
                        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(rb64 >> 32));
                        mine = __longlong_as_double(((unsigned long long)hi << 32) | lo);
                    }
                    if (kh == 0 && valid[h]) {
                        // the reference view itself is no V entry (MVS2.py:66-67)
                        const uint64_t self = (mk >> Rv[h]) & 1ull;
                        mk &= ~(1ull << Rv[h]);
                        const int cnt = __popcll(mk);
                        const int64_t idx = e[h].x;
                        a.mask[idx * a.mstride] = mk;
                        if (a.count) a.count[idx] = cnt;
                        if (a.avg) {
                            // its own term num_RR w_a = D_a w_a = sqrt(D_a) = 1 / w_a (to
                            // the rsq + Newton accuracy of w_a, 4e-15) leaves the sum
                            double inv = __builtin_amdgcn_rcp(my_wa[h]);
                            inv = inv * (2.0 - my_wa[h] * inv);
                            const double sum = self ? mine - inv : mine;
                            a.avg[idx * a.astride] = cnt ? sum * (kn * my_wa[h]) * s_recip[cnt] : 0.0;
                        }
                        if (gg) {
                            t.fix_list[atomicAdd(t.fix_count, 1)] = make_int4((int32_t)idx, dcur.x, e[h].y, 0);
                            STAMP_ADD_ANY(11, 1);
                        }
                    }
                }
    #ifdef MVS_STAMPS
                STAMP_ADD_LANE0(12, span > KSK ? 1 : 0);
                STAMP_ADD_LANE0(13, 1);
    #endif
              };
              if (nh == 2) unit(std::integral_constant<int, 2>{});
              else unit(std::integral_constant<int, 1>{});
            }
            STAMP(t3);
    #ifdef MVS_STAMPS
            // slowest wave's own phase-3 time (per item: slot 9), every wave's (10)
            if (lane == 0) atomicMax(&s_maxown, (unsigned)(t3 - t2));
            STAMP_ADD_LANE0(10, t3 - t2);
    #endif
            __syncthreads();
            STAMP(t4);
            STAMP_ADD(0, 1);
            STAMP_ADD(1, t1 - t0);
            STAMP_ADD(2, t2 - t1);
            STAMP_ADD(3, t4 - t2);
            STAMP_ADD_W0(4, t3 - t2);
            STAMP_ADD_W0(5, w0blk);
            STAMP_ADD(6, t1a - t1);
            STAMP_ADD(7, t1b - t1a);
            STAMP_ADD_W0(8, t4 - t3);
    #ifdef MVS_STAMPS
            if (tid == 0) {
                STAMP_ADD_ANY(9, s_maxown);
                s_maxown = 0;
            }
    #endif
        if (nx1 >= n_units) return false;
        if constexpr (!DB) stage(dnx1, std::integral_constant<int, 0>{});   // the buffer is free now; lands by the next barrier
        cur = nx1;
        dcur = dnx1;
        nx1 = nx2;
        dnx1 = dnx2;
        return true;
    };
    for (;;) {
        if (!round(std::integral_constant<int, 0>{})) break;
        if (!round(std::integral_constant<int, DB ? 1 : 0>{})) break;
    }
}

// ---------------------------------------------------------------------------
// k_score_mma_v (64 < V <= 256): the views in groups of 64 (one mask word
// each).  A workgroup takes one work item (the candidates of one 16x8 tile,
// at most kGroupChunk of them) from the queue and scores it against every
// view group in turn:
//   0. (per item) the candidate list is sorted by the candidate's row in the
//      tile (counting sort over 8 rows), so that an M-block of 16 candidates
//      spans few region rows and its K-loop skips the K-steps none of its
//      windows reaches;
//   1. (per item) each candidate's own reference window rows go to LDS by
//      LDS-DMA (its view is usually in another group); behind group 0's
//      phase 2 they are masked in place to the window's columns (the A
//      operands need no masking afterwards), S_a and S_aa summed per row by
//      every thread, and the decision constants derived;
//   2. (per group) Q = S_bb of every (pixel, view) of the group (int32; -1
//      past V): one thread per (pixel column, view) sums its column's window
//      rows straight from the staged region (masked v_dot4_i32_i8) and slides
//      them down the tile;
//   3. (per group) wave tasks (M-block of 16 candidates, 32 views): C = sum
//      s_R s_v and S_b = sum s_v over the window, both by
//      v_mfma_i32_16x16x64_i8 (S_b with the window's 0/1 indicator row as A,
//      from a 16-entry table by the window's column); D = n Q - S_b^2 and
//      num = n C - S_a S_b (24-bit multiplies: |S_b| < 2^14, Q < 2^21); the
//      decision num w_b > T in binary32 with w_b = v_rsq_f32(D) (guard band
//      2e-6 |T| as in k_score_mma; D = 0, a constant window, gives
//      0 * inf = nan and never passes), the sum of the passing num w_b with
//      w_b refined in binary64 (one Newton step);
//   4. (per group) each candidate's mask word, count, sum and guard flag
//      accumulate in its thread's registers; written after the last group
//      (guard-band candidates to k_score_fix).
// The regions are double-buffered: group k+1's (after an item's last group,
// the next item's first) lands by LDS-DMA while group k is scored, as do the
// next item's candidate list and, behind group 0's phase 2, an item's
// reference rows.  Every LDS-DMA target is a static LDS array of its own, so
// that the compiler sees no aliasing with the tables phases 2-4 read and
// write.  Work items come in tile order (k_item_scan): the workgroups in flight
// share image rows, so TLB and L2 reach over 256 views of a large image.
// ---------------------------------------------------------------------------
constexpr int kVTab = 68;   // Q-table row pitch (int32): the per-column writes are conflict free

// a candidate's constants (LDS, per item)
struct alignas(16) CandInfoV {
    int32_t px, R, Sa, pk;    // Q-table row of its pixel (px * kVTab), reference view, -S_a, packed pixel
    float T, gT;              // decision threshold on num w_b and its guard band
    double ca;                // n / (n-1) * w_a
};

// dynamic LDS of k_score_mma_v (the LDS-DMA targets are static arrays)
struct VLds {
    int qtab, ci, rmask, rguard, rsum, total;
};

template <bool TAB>
__host__ __device__ constexpr VLds v_lds() {
    VLds L{};
    L.qtab = 0;                                                 // [128 px][kVTab] int32 (TAB: none)
    L.ci = L.qtab + (TAB ? 0 : 128 * kVTab * 4);
    L.rmask = L.ci + kGroupChunk * (int)sizeof(CandInfoV);      // [cand][4 view blocks] u16 (item start:
                                                                // [cand] {S_a, S_aa} int32 sums)
    L.rguard = L.rmask + kGroupChunk * 4 * 2;                   // [cand][2 halves] u16
    L.rsum = L.rguard + kGroupChunk * 2 * 2 + 8;                // [cand][2 halves] double (8-B aligned)
    L.total = L.rsum + kGroupChunk * 2 * 8;
    return L;
}

template <int WID>
__host__ __device__ constexpr int v_static_lds() {
    return 2 * 64 * MmaGeom<WID>::VS + 2 * kGroupChunk * 8 + kGroupChunk * MmaGeom<WID>::NB * 32 + 16 +
           16 * 32 + 16 + 16 + 16 * 4;
}


// byte masks of a window of NB bytes starting at byte b0 over the 4 dwords
// from dword b0 >> 2
template <int NB>
DEV void window_dword_masks(int b0, uint32_t (&mk)[4]) {
    const int e = b0 + NB;   // one past the last byte
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int base = 4 * ((b0 >> 2) + j);
        const int lo = max(b0 - base, 0), n = min(e - base, 4) - lo;   // bytes [lo, lo + n) of dword j
        mk[j] = n > 0 ? (uint32_t)(((1ull << (8 * n)) - 1ull) << (8 * lo)) : 0u;
    }
}

// 1/sqrt(D) in binary64: v_rsq_f64 + one Newton step (max relative error
// 4.1e-15 over 4M values of D < 2^31, tools/ubench/rsq_acc.hip); nan for D <= 0
DEV double rsqrt_nr(int D) {
    double w = __builtin_nan("");
    if (D > 0) {
        const double x = (double)D;
        w = __builtin_amdgcn_rsq(x);
        w = w * (1.5 - 0.5 * x * w * w);
    }
    return w;
}

template <int WID, bool FAST, bool TAB>
__global__ __launch_bounds__(kMmaThreads) void k_score_mma_v(const SceneDev sc, const ScoreArgs a, const TiledArgs t,
                                                             const MomentsDev mt, const int4* __restrict__ items,
                                                             const int2* __restrict__ sorted) {
    using G = MmaGeom<WID>;
    constexpr int NB = G::NB, NPX = G::NPX, ROWS = G::ROWS, VS = G::VS, C0 = G::C0;
    constexpr int RPV = VS / 32;
    constexpr int NPIECE = 64 * RPV * 2;                                              // 16-B pieces of a region
    constexpr int RPIECE = (NPIECE + kMmaThreads - 1) / kMmaThreads;                  // ... per thread
    constexpr int APIECE = (kGroupChunk * NB * 2 + kMmaThreads - 1) / kMmaThreads;   // reference-row pieces
    constexpr int AROW = (kGroupChunk * NB + kMmaThreads - 1) / kMmaThreads;         // reference rows per thread
    static_assert(kGroupChunk <= 128, "one phase-3 task per wave; the sort ranks two waves");
    // LDS-DMA targets: two regions, the candidate list as it lands (s_cd0) and
    // sorted by row (s_cd1), the reference rows
    __shared__ __attribute__((aligned(16))) uint8_t s_rg0[64 * VS], s_rg1[64 * VS];
    __shared__ __attribute__((aligned(16))) uint8_t s_cd0[kGroupChunk * 8], s_cd1[kGroupChunk * 8];
    // the reference rows, then 16 zero bytes (never an LDS-DMA target): phase
    // 3 reads a row or the zeros through an offset select inside the one
    // array, so that the read carries the array's alias scope and waits for
    // no LDS-DMA in flight (a select between two arrays would wait for all)
    constexpr int AZERO = kGroupChunk * NB * 32;
    __shared__ __attribute__((aligned(16))) uint8_t s_areg[AZERO + 16];
    // the window indicator rows by window column (0/1 bytes), then 16 zeros
    __shared__ __attribute__((aligned(16))) uint8_t s_ind[16 * 32 + 16];
    __shared__ int s_item;
    __shared__ __attribute__((aligned(16))) int32_t s_cnt[16];   // the sort's per-wave row counts
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr VLds L = v_lds<TAB>();
    const int16_t* __restrict__ tsb = mt.sb;   // TAB: S_b and D = n S_bb - S_b^2 per (pixel, view)
    const int32_t* __restrict__ tdd = mt.d;
    const int VPt = mt.VP;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int V = sc.V;
    const int NG = t.groups;
    int32_t* qtab = (int32_t*)(smem + L.qtab);
    CandInfoV* ci = (CandInfoV*)(smem + L.ci);
    uint16_t* rmask = (uint16_t*)(smem + L.rmask);
    int32_t* asums = (int32_t*)(smem + L.rmask);   // item start only: {S_a, S_aa} per candidate
    uint16_t* rguard = (uint16_t*)(smem + L.rguard);
    double* rsum = (double*)(smem + L.rsum);
    const double kn = (double)NPX / (double)(NPX - 1);
    const float tqf = (float)(a.thr / kn);
    ItemMap im;
    im.load(t);
    const int n_items = im.total();
    int32_t* head = t.head;

    // region piece k (view k / 2RPV, row, half) of view group g at a tile: its
    // gv address; rows outside the image are clamped (their pixels are never
    // in a valid window), views past V repeat the last (never used)
    auto region_src = [&](int tile, int g, int k) -> const uint8_t* {
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int v = k / (2 * RPV), r2 = k - v * (2 * RPV);
        const int y = min(max(ty * MVS_TILE_H - WID + (r2 >> 1), 0), sc.H - 1);
        const int view = min(g * 64 + v, V - 1);
        return sc.gv + ((int64_t)view * sc.H + y) * sc.Wp + (tx * MVS_TILE_W - 8) + 16 * (r2 & 1);
    };
    auto stage_region = [&](int tile, int g, auto bufc) {
        uint8_t* dst = decltype(bufc)::value ? s_rg1 : s_rg0;
        const int tv = opaque(tid);   // per-lane addressing recomputed here, not held across the loop
#pragma unroll
        for (int p = 0; p < RPIECE; ++p) {
            const int k = tv + p * kMmaThreads;
            if (k < NPIECE)
                __builtin_amdgcn_global_load_lds((const void*)region_src(tile, g, k),
                                                 (void __attribute__((address_space(3)))*)(dst + (p * kMmaThreads + wave * 64) * 16),
                                                 16, 0, 0);
        }
    };
    // an item's candidate list always lands in s_cd0 (free once sorted into s_cd1)
    auto stage_cands = [&](const int4 d) {
        const int32_t* csrc = (const int32_t*)(sorted + d.y);
        if (tid < 2 * d.z)
            __builtin_amdgcn_global_load_lds((const void*)(csrc + tid),
                                             (void __attribute__((address_space(3)))*)(s_cd0 + wave * 64 * 4),
                                             4, 0, 0);
    };

    // the items in contiguous bands of tiles, band x claimed first by the
    // workgroups b = x mod kBandHeads (one band per XCD under round-robin
    // dispatch: an XCD's workgroups in flight take neighbouring tiles and
    // share their regions' lines in its L2; ring256 0.498 vs 0.506 ms with
    // one queue, profiles/r06/r6n_*)
    const int ob = (int)blockIdx.x % kBandHeads;
    int cb = ob;   // thread 0's current band
    auto claim_item = [&]() -> int {
        return band_claim(head + (3 + kItemSegs) * 32, cb, ob, kBandHeads, n_items, [](int) { return 0; });
    };
    // the first item: its candidates and group 0's region; the indicator rows
    if (tid == 0) s_item = claim_item();
    if (tid < 16 * 8) {   // indicator row q: bytes [q + C0, q + C0 + NB) are 1
        const int q = tid >> 3, j = tid & 7;
        const uint32_t wm = ((1u << NB) - 1u) << (q + C0);
        ((uint32_t*)s_ind)[tid] = byte_mask((wm >> (4 * j)) & 15u) & 0x01010101u;
    } else if (tid < 16 * 8 + 4) {
        ((uint32_t*)(s_ind + 16 * 32))[tid - 16 * 8] = 0u;
        ((uint32_t*)(s_areg + AZERO))[tid - 16 * 8] = 0u;
    }
    __syncthreads();
    int item = __builtin_amdgcn_readfirstlane(s_item);
    if (item >= n_items) return;
    int4 d = item_desc(t, items, im, item);
    stage_cands(d);
    stage_region(d.x, 0, std::integral_constant<int, 0>{});
    __syncthreads();
    int kpar = 0;    // region buffer of this group (groups alternate across items)

    for (;;) {
        const int tile = d.x, nc = d.z;
        const int ty = tile / t.ntx;
        const int x0 = (tile - ty * t.ntx) * MVS_TILE_W;
        const int2* cand = (const int2*)s_cd1;
        // ---- 0. the candidates sorted by row (counting sort, two waves) ----
        {
            const int2 e = tid < nc ? ((const int2*)s_cd0)[tid] : make_int2(0, 0);
            const int key = (e.y >> 4) & 7;
            int rank = 0;
            if (wave < 2) {
                int cntv = 0;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const uint64_t m = __ballot(tid < nc && key == r);
                    if ((tid & 63) == r) cntv = __popcll(m);
                    if (key == r) rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                }
                if ((tid & 63) < 8) s_cnt[wave * 8 + (tid & 63)] = cntv;
            }
            if (tid < 2 * kGroupChunk) asums[tid] = 0;
            lds_barrier();
            if (tid < nc) {
                int pos = rank;
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const int c0 = s_cnt[r], c1 = s_cnt[8 + r];
                    pos += (r < key ? c0 + c1 : 0) + (r == key && wave == 1 ? c0 : 0);
                }
                ((int2*)s_cd1)[pos] = e;
            }
            lds_barrier();
        }
        const int my_idx = tid < nc ? cand[tid].x : 0;
        // ---- 1. the candidates' reference rows (they land behind phase 2) ----
        // (the candidate entries are read first: an LDS read between two
        // LDS-DMA issues would wait for the first)
        const int tv = opaque(tid);
        int pks[APIECE];
#pragma unroll
        for (int p = 0; p < APIECE; ++p) {
            const int k = tv + p * kMmaThreads;
            pks[p] = k < nc * NB * 2 ? cand[k / (2 * NB)].y : 0;
        }
#pragma unroll
        for (int p = 0; p < APIECE; ++p) {
            const int k = tv + p * kMmaThreads;
            if (k < nc * NB * 2) {
                const int kk = k / (2 * NB), r2 = k - kk * (2 * NB);
                const int pk = pks[p];
                const int y = ty * MVS_TILE_H + ((pk >> 4) & 7) - WID + (r2 >> 1);   // inside: the window is valid
                const uint8_t* src = sc.gv + ((int64_t)(pk >> 7) * sc.H + y) * sc.Wp + (x0 - 8) + 16 * (r2 & 1);
                __builtin_amdgcn_global_load_lds((const void*)src,
                                                 (void __attribute__((address_space(3)))*)(s_areg + (p * kMmaThreads + wave * 64) * 16),
                                                 16, 0, 0);
            }
        }

        int next = n_items;
        int4 dn = make_int4(0, 0, 0, 0);
        int acnt = 0;
        double asum = 0.0;
        uint32_t aguard = 0;
        uint64_t pend = 0;   // the previous group's mask word, stored during this group's phase 2

        // one view group; its region is in s_rg<buf>
        auto group = [&](const int g, auto bufc) {
            constexpr int buf = decltype(bufc)::value;
            // the per-lane maps, recomputed per group rather than held in
            // registers across the item loop
            const int tid = opaque(threadIdx.x), lane = tid & 63;
            const int m = lane & 15, kh = lane >> 4;
            // phase 2 map: thread = (pixel column mx, view mv); 16 columns x 4 views per wave
            const int mx = tid & 15, mv = tid >> 4;
            uint32_t cmk[4];
            window_dword_masks<NB>(mx + C0, cmk);
            const int cd0 = (mx + C0) >> 2;
            const uint8_t* reg = buf ? s_rg1 : s_rg0;
            STAMP(t0);
            const int vb = g * 64;
            const int GV = min(64, V - vb);
            const bool last = g + 1 == NG;
            // the next region (group g+1, or the next item's group 0) and, after
            // the last group, the next item's candidates land during phases 3-4
            auto prefetch = [&]() {
                if (!last) {
                    stage_region(tile, g + 1, std::integral_constant<int, buf ^ 1>{});
                } else if (next < n_items) {
                    stage_cands(dn);
                    stage_region(dn.x, 0, std::integral_constant<int, buf ^ 1>{});
                }
            };
            // group 0: thread 0 claims the next item; the result is in by the
            // barrier after phase 2, which waits for the reference rows anyway
            // (claimed inside the group loop: a VGPR loaded before the loop and
            // read in it would make the compiler drain every load at loop entry)
            int claim = 0;
            if (g == 0 && tid == 0) claim = claim_item();
            // ---- 2. Q = S_bb of every (pixel, view) of the group ----
            // (TAB: none, the scene's tables hold S_b and D)
            if (TAB) {
            } else if (mv < GV) {
                // rows in order, the window sliding down as they come: at most
                // NB + 1 row sums live
                int Q[ROWS];
                const uint8_t* col = reg + mv * VS + 4 * cd0;
                int q = 0;
#pragma unroll
                for (int rho = 0; rho < ROWS; ++rho) {
                    int qr = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int dm = (int)(*(const uint32_t*)(col + rho * 32 + 4 * j) & cmk[j]);
                        qr = __builtin_amdgcn_sdot4(dm, dm, qr, false);
                    }
                    Q[rho] = qr;
                    q += qr;
                    if (rho >= NB) q -= Q[rho - NB];
                    if (rho >= NB - 1) qtab[((rho - (NB - 1)) * 16 + mx) * kVTab + mv] = q;
                }
            } else {
#pragma unroll
                for (int y = 0; y < MVS_TILE_H; ++y) qtab[(y * 16 + mx) * kVTab + mv] = -1;   // D < 0: nan
            }
            (void)mx; (void)mv; (void)cmk; (void)cd0;
            STAMP(t0a);
            // (and, group 0, the reference rows have landed; nothing else is in
            // flight, so the LDS reads of phases 3-4 need no waits)
            __syncthreads();
            STAMP(t0b);
            if (g == 0) {
                if (tid == 0) s_item = claim;   // published by the barriers below
                // the reference rows masked in place to their window's columns,
                // and their sums: one thread per (candidate, row)
#pragma unroll
                for (int p = 0; p < AROW; ++p) {
                    const int k = tid + p * kMmaThreads;
                    if (k < nc * NB) {
                        const int qrel = cand[k / NB].y & 15;
                        const uint32_t wm = ((1u << NB) - 1u) << (qrel + C0);
                        uint4* row = (uint4*)(s_areg + k * 32);
                        uint4 h0 = row[0], h1 = row[1];
                        h0.x &= byte_mask(wm & 15u);
                        h0.y &= byte_mask((wm >> 4) & 15u);
                        h0.z &= byte_mask((wm >> 8) & 15u);
                        h0.w &= byte_mask((wm >> 12) & 15u);
                        h1.x &= byte_mask((wm >> 16) & 15u);
                        h1.y &= byte_mask((wm >> 20) & 15u);
                        h1.z &= byte_mask((wm >> 24) & 15u);
                        h1.w &= byte_mask(wm >> 28);
                        row[0] = h0;
                        row[1] = h1;
                        int s = 0, q = 0;
                        const uint32_t dw[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            s = __builtin_amdgcn_sdot4((int)dw[j], 0x01010101, s, false);
                            q = __builtin_amdgcn_sdot4((int)dw[j], (int)dw[j], q, false);
                        }
                        atomicAdd(&asums[2 * (k / NB)], s);
                        atomicAdd(&asums[2 * (k / NB) + 1], q);
                    }
                }
                lds_barrier();
                // the candidates' constants
                if (tid < nc) {
                    const int pk = cand[tid].y;
                    const int s = asums[2 * tid], q = asums[2 * tid + 1];
                    const double wa = rsqrt_nr(NPX * q - s * s);
                    CandInfoV c;
                    // the pixel's row: of the Q table, or (TAB) of the scene's tables
                    c.px = TAB ? ((ty * MVS_TILE_H + ((pk >> 4) & 7)) * sc.W + x0 + (pk & 15)) * VPt
                               : (pk & 127) * kVTab;
                    c.R = pk >> 7;
                    c.Sa = -s;
                    c.pk = pk;
                    c.T = tqf * __builtin_amdgcn_rcpf((float)wa);   // nan for a constant window
                    c.gT = 2e-6f * fabsf(c.T);
                    c.ca = kn * wa;
                    ci[tid] = c;
                }
                lds_barrier();
                next = __builtin_amdgcn_readfirstlane(s_item);
                if (next < n_items) dn = item_desc(t, items, im, next);
            }
            STAMP(t1);
            prefetch();
            // the previous group's mask word: its store has phases 3-4 to complete
            // (the barrier after phase 4 waits for it with the region's LDS-DMA)
            if (g > 0 && tid < nc) a.mask[(int64_t)my_idx * a.mstride + g - 1] = pend;
            asm volatile("" ::: "memory");   // the LDS-DMA issues stay ahead of phase 3
            STAMP(tpf);

            // ---- 3. wave task (M-block b, views 32 h + [0, 32)) ----
            const int nblk = (nc + 15) >> 4;
            if (wave < nblk * 2) {
                const int b = wave >> 1, h = wave & 1;
                const int kk = b * 16 + m;
                const bool valid = kk < nc;
                const int pk = valid ? ci[kk].pk : 0;
                const int qrel = pk & 15, rrel = (pk >> 4) & 7;
                // the block's rows (sorted): K-steps s0..s1 hold every window row
                const int r_lo = __builtin_amdgcn_readfirstlane((ci[b * 16].pk >> 4) & 7);
                const int r_hi = __builtin_amdgcn_readfirstlane((ci[min(b * 16 + 15, nc - 1)].pk >> 4) & 7);
                const int s0 = r_lo >> 1, s1 = (r_hi + NB - 1) >> 1;
                const int lofs = 32 * (kh >> 1) + 16 * (kh & 1);
                // region row 2s + (kh >> 1) = window row 2s + (kh >> 1) - rrel of the candidate
                const int aoff = (min(kk, nc - 1) * NB - rrel) * 32 + 16 * (kh & 1);
                const int ioff = qrel * 32 + 16 * (kh & 1);
                const uint8_t* bptr0 = reg + min(32 * h + m, GV - 1) * VS + lofs;
                const uint8_t* bptr1 = reg + min(32 * h + 16 + m, GV - 1) * VS + lofs;
                v4i C0v = {0, 0, 0, 0}, C1v = {0, 0, 0, 0}, S0v = {0, 0, 0, 0}, S1v = {0, 0, 0, 0};
                auto kstep = [&](const int s) {
                    const int row = 2 * s + (kh >> 1);
                    const bool rv = valid && row >= rrel && row < rrel + NB;
                    // rows outside the window read 16 zero bytes: an offset select
                    // instead of a branch around the load
                    const uint4 av = *(const uint4*)(s_areg + (rv ? aoff + row * 32 : AZERO));
                    const uint4 iv = *(const uint4*)(s_ind + (rv ? ioff : 16 * 32));
                    const v4i AI = {(int)iv.x, (int)iv.y, (int)iv.z, (int)iv.w};
                    const v4i A = {(int)av.x, (int)av.y, (int)av.z, (int)av.w};
                    const uint4 b0 = *(const uint4*)(bptr0 + 64 * s);
                    const uint4 b1 = *(const uint4*)(bptr1 + 64 * s);
                    const v4i B0 = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w};
                    const v4i B1 = {(int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
                    C0v = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B0, C0v, 0, 0, 0);
                    C1v = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B1, C1v, 0, 0, 0);
                    if constexpr (!TAB) {
                        S0v = __builtin_amdgcn_mfma_i32_16x16x64_i8(AI, B0, S0v, 0, 0, 0);
                        S1v = __builtin_amdgcn_mfma_i32_16x16x64_i8(AI, B1, S1v, 0, 0, 0);
                    } else {
                        (void)AI;
                    }
                };
                // every window takes KMIN K-steps: those unrolled from sb (loads
                // issued ahead of the MFMAs), the block's further ones after
                constexpr int KMIN = (NB + 2) / 2;
                const int sb = min(s0, G::KS - KMIN);
#pragma unroll
                for (int u = 0; u < KMIN; ++u) kstep(sb + u);
                for (int s = sb + KMIN; s <= s1; ++s) kstep(s);
                // lane (kh, m) holds candidate 16 b + 4 kh + i, views vb + 32 h + 16 j + m
                uint32_t pmv = 0, gdv = 0;
                double sacc[4];
                // TAB: S_b and D of candidate 4 kh + i's pixel at views vb + 32 h +
                // 16 j + m from the tables, one candidate step ahead of their use
                int tsbv[2][2], tdv[2][2];
                auto tfetch = [&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    if constexpr (TAB) {
                        const int px = ci[min(b * 16 + 4 * kh + i, nc - 1)].px + vb + 32 * h + m;
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            tsbv[i & 1][j] = tsb[px + 16 * j];
                            tdv[i & 1][j] = tdd[px + 16 * j];
                        }
                    }
                };
                tfetch(std::integral_constant<int, 0>{});
                static_for<4>([&](auto Ic) {
                    constexpr int i = Ic;
                    if constexpr (i < 3) tfetch(std::integral_constant<int, i + 1>{});
                    const CandInfoV c = ci[min(b * 16 + 4 * kh + i, nc - 1)];
                    double sa = 0.0;
                    uint64_t gacc = 0;
                    static_for<2>([&](auto Jc) {
                        constexpr int j = Jc;
                        const int vl = 32 * h + 16 * j + m;
                        const int Sb = TAB ? tsbv[i & 1][j] : (j ? S1v[i] : S0v[i]);
                        const int D = TAB ? tdv[i & 1][j]
                                          : __mul24(NPX, qtab[c.px + vl]) - __mul24(Sb, Sb);   // < 0 past V: nan
                        const float wf = __builtin_amdgcn_rsqf((float)D);
                        const int num = __mul24(c.Sa, Sb) + __mul24(NPX, j ? C1v[i] : C0v[i]);
                        const uint64_t liv = __builtin_amdgcn_uicmp((uint32_t)(vb + vl), (uint32_t)c.R, 33);
                        // w_b in binary64: one Newton step from the binary32 estimate
                        double w = (double)wf;
                        w = w * (1.5 - 0.5 * (double)D * w * w);
                        uint64_t P, Gd;
                        if constexpr (FAST) {
                            const float x = fmaf((float)num, wf, -c.T);
                            P = __builtin_amdgcn_fcmpf(x, 0.0f, 2) & liv;
                            Gd = __builtin_amdgcn_fcmpf(fabsf(x), c.gT, 4) & liv;
                        } else {
                            const double ncc = (double)num * w * c.ca;
                            P = __ballot(vb + vl != c.R && ncc > a.thr);
                            Gd = __ballot(vb + vl != c.R && fabs(ncc - a.thr) <= kGuard);
                        }
                        pmv = writelane<2 * (2 * i + j)>(pmv, (uint32_t)P);
                        pmv = writelane<2 * (2 * i + j) + 1>(pmv, (uint32_t)(P >> 32));
                        gacc |= Gd;
                        sa = fma_f64_lanes(sa, num, w, P);
                    });
                    gdv = writelane<2 * i>(gdv, (uint32_t)gacc);
                    gdv = writelane<2 * i + 1>(gdv, (uint32_t)(gacc >> 32));
                    sacc[i] = sa;
                    __builtin_amdgcn_sched_barrier(0);   // one candidate row at a time: register pressure
                });
                // candidate 16 b + l (l = 4 q + i): 16-bit piece q of ballot (i, j)
                {
                    const int l = lane & 15, i = l & 3, q = l >> 2;
                    const int cc = b * 16 + l;
                    uint32_t pc[2];
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const uint32_t lo = __builtin_amdgcn_ds_bpermute(4 * (2 * (2 * i + j)), (int)pmv);
                        const uint32_t hi = __builtin_amdgcn_ds_bpermute(4 * (2 * (2 * i + j) + 1), (int)pmv);
                        pc[j] = (uint32_t)(((((uint64_t)hi << 32) | lo) >> (16 * q)) & 0xffffu);
                    }
                    const uint32_t glo = __builtin_amdgcn_ds_bpermute(4 * (2 * i), (int)gdv);
                    const uint32_t ghi = __builtin_amdgcn_ds_bpermute(4 * (2 * i + 1), (int)gdv);
                    const uint32_t gq = (uint32_t)(((((uint64_t)ghi << 32) | glo) >> (16 * q)) & 0xffffu);
                    if (lane < 16 && cc < nc) {
                        ((uint32_t*)rmask)[cc * 2 + h] = pc[0] | (pc[1] << 16);
                        rguard[cc * 2 + h] = (uint16_t)gq;
                    }
                }
                if (a.avg != nullptr) {
                    const double mine = row_sum16_x4(sacc, m);
                    const int cc = b * 16 + 4 * kh + m;
                    if (m < 4 && cc < nc) rsum[cc * 2 + h] = mine;
                }
            }
            STAMP(t1a);
            lds_barrier();
            STAMP(t2);
            // ---- 4. the group's mask word, count, sum and guard accumulate ----
            if (tid < nc) {
                const uint64_t mk = *(const uint64_t*)(rmask + tid * 4);   // views 16 nb + [0, 16) at bits 16 nb
                aguard |= rguard[tid * 2] | rguard[tid * 2 + 1];
                pend = mk;
                acnt += __popcll(mk);
                if (a.avg != nullptr && mk) asum += (rsum[tid * 2] + rsum[tid * 2 + 1]) * ci[tid].ca;
            }
            __syncthreads();   // the next region has landed
            STAMP(t3);
            STAMP_ADD(0, 1);
            STAMP_ADD(1, t1 - t0);
            STAMP_ADD(2, t2 - t1);
            STAMP_ADD(3, t3 - t2);
            STAMP_ADD(4, t0a - t0);    // wave 0: phase 2 own work
            STAMP_ADD(5, t0b - t0a);   // barrier after phase 2 (group 0: the reference rows)
            STAMP_ADD(6, t1 - t0b);    // group 0: the candidate constants
            STAMP_ADD(7, t1a - t1);    // wave 0: prefetch issue + its phase-3 task
            if (g == 0) STAMP_ADD(8, t0b - t0a);                     // barrier after phase 2, group 0 only
            STAMP_ADD_LANE0(9, t0a - t0);                            // every wave's own phase-2 work
            STAMP_ADD(10, tpf - t1);                                 // wave 0: prefetch + mask-store issue
            if (wave < ((nc + 15) >> 4) * 2) {
                STAMP_ADD_LANE0(11, t1a - tpf);                      // a task's phase-3 time (waves with tasks)
                STAMP_ADD_LANE0(12, 1);                              // tasks
            }
        };
        for (int g = 0; g < NG; ++g) {
            if (kpar) group(g, std::integral_constant<int, 1>{});
            else group(g, std::integral_constant<int, 0>{});
            kpar ^= 1;
        }
        if (tid < nc) {
            a.mask[(int64_t)my_idx * a.mstride + NG - 1] = pend;
            if (a.count) a.count[my_idx] = acnt;
            if (a.avg) a.avg[(int64_t)my_idx * a.astride] = acnt ? asum * (1.0 / (double)acnt) : 0.0;
            if (aguard) t.fix_list[atomicAdd(t.fix_count, 1)] = make_int4(my_idx, tile, cand[tid].y, 0);
        }
        if (next >= n_items) break;
        item = next;
        d = dn;
    }
}

// Guard-band candidates of the tiled scorer and bucket overflow, re-scored
// whole by the direct path (whose own guard band leads to the numpy-order
// ctNcc).  Last kernel of a batch.  It zeroes nothing: the tile counters and
// the control block come in two parity sets, and the next batch's k_bin
// zeroes this batch's set (no done ticket here: a kernel with a short list
// is a launch and one load: 6.8 -> 4.7 us with 30 guard-band entries,
// profiles/r06/r6p_*).  The grid has kFixBase workgroups plus, for large batches, more that take
// part only when the list is long (a skewed batch whose tiles overflow their
// buckets): a guard-band list of a few hundred entries costs no extra
// workgroups' atomics, a long overflow list gets up to 4x the workgroups.
constexpr int kFixBase = 64, kFixSmall = kFixBase * 4 * 8;

template <int WID, int NS>
__global__ __launch_bounds__(256) void k_score_fix(const SceneDev sc, const ScoreArgs a,
                                                   const TiledArgs t) {
    const int nfix = *t.fix_count;
    if (blockIdx.x == 0 && threadIdx.x == 0 && t.stats) {
        t.stats[0] += (unsigned long long)nfix;
        t.stats[2] += 1ull;
    }
    const int active = nfix > kFixSmall ? (int)gridDim.x : kFixBase;   // uniform over the grid
    if ((int)blockIdx.x >= active) return;
    for (int k = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); k < nfix;
         k += active * 4) {
        const int4 f = t.fix_list[k];
        const int64_t cand = __builtin_amdgcn_readfirstlane(f.x);
        const int tile = __builtin_amdgcn_readfirstlane(f.y);
        const int pk = __builtin_amdgcn_readfirstlane(f.z);
        const int ty = tile / t.ntx, tx = tile - ty * t.ntx;
        const int q = tx * MVS_TILE_W + (pk & 15), r = ty * MVS_TILE_H + ((pk >> 4) & 7), R = pk >> 7;
        wave_score<WID, NS>(sc, R, q, r, a.thr, a.mask + cand * a.mstride, a.count ? a.count + cand : nullptr,
                            a.avg ? a.avg + cand * a.astride : nullptr, a.exact_hits);
    }
}

// ---------------------------------------------------------------------------
// patch_expansion children (MVS2.py:329-369)
// ---------------------------------------------------------------------------
DEV double dot3(const double* a, const double* b) {
    // np.dot of two float64 3-vectors as OpenBLAS 0.3.29 evaluates it.
    return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]));
}

DEV int py_wrap(int i, int n) { return i < 0 ? i + n : i; }

// Geometry of child k: ray through the (buggy) cell centre, intersection
// with the parent's plane, normal, colour, projection into the child's own
// view and its cell; written into the child's record row `out`.
DEV void child_geometry(const SceneDev& sc, const RecordsDev& rec, const ExpandArgs& a, const ChildJob job,
                        int64_t out, double* X, double* nX, double* pxo, double* pyo) {
    const int64_t par = job.parent;
    const int v = job.view;
    const int di = job.di;
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
#pragma unroll
    for (int j = 0; j < 3; ++j) X[j] = cm.O[j] + tt * d[j];
    const double e0 = X[0] - cm.O[0], e1 = X[1] - cm.O[1], e2 = X[2] - cm.O[2];
    const double dist = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
#pragma unroll
    for (int j = 0; j < 3; ++j) nX[j] = (cm.O[j] - X[j]) / dist;
    double px, py;
    project(cm, X, px, py);
    *pxo = px;
    *pyo = py;
}

DEV void child_write(const SceneDev& sc, const RecordsDev& rec, const ExpandArgs& a, const ChildJob job,
                     int64_t out, const double* X, const double* nX, double px, double py) {
    const int v = job.view;
    const double cs = (double)a.cell_size;
    const int64_t par = job.parent;
    const double ci = floor(rec.xy[2 * par] / cs), cj = floor(rec.xy[2 * par + 1] / cs);
    const double cc0 = cs * ((ci + job.di) + 0.5);
    const double cc1 = cs * ((cj + job.di) + 0.5);
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

// accept test (MVS2.py:369) with is_patch_neighbor (MVS2.py:298-299)
DEV uint8_t child_accept(const RecordsDev& rec, const ExpandArgs& a, int64_t par, const double* X,
                         const double* nX, int cnt) {
    const double pc[3] = {rec.c[3 * par], rec.c[3 * par + 1], rec.c[3 * par + 2]};
    const double pn[3] = {rec.n[3 * par], rec.n[3 * par + 1], rec.n[3 * par + 2]};
    const double pm[3] = {pc[0] - X[0], pc[1] - X[1], pc[2] - X[2]};
    const double nb = fabs(dot3(pm, pn) + dot3(pm, nX));
    const double g0 = pc[0] - X[0], g1 = pc[1] - X[1], g2 = pc[2] - X[2];
    const double dd = sqrt((g0 * g0 + g1 * g1) + g2 * g2);
    return (cnt >= a.vlb && nb < 0.1 && dd < a.dist_thr) ? 1 : 0;
}

// one wave per child: geometry, direct photo test, accept test (small sweeps)
template <int WID, int NS>
__global__ __launch_bounds__(256) void k_expand(const SceneDev sc, RecordsDev rec, const ExpandArgs a) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= a.n) return;
    const int lane = threadIdx.x & 63;
    const int words = (sc.V + 63) >> 6;
    const ChildJob job = a.jobs[k];
    const int v = __builtin_amdgcn_readfirstlane((int)job.view);
    const int64_t out = a.first_out + k;
    double X[3], nX[3], px, py;
    child_geometry(sc, rec, a, job, out, X, nX, &px, &py);
    if (lane == 0) child_write(sc, rec, a, job, out, X, nX, px, py);
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
    if (lane == 0) rec.accept[out] = child_accept(rec, a, job.parent, X, nX, rec.count[out]);
}

// large sweeps: one thread per child for the geometry ...
__global__ void k_expand_geom(const SceneDev sc, RecordsDev rec, const ExpandArgs a) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const ChildJob job = a.jobs[k];
        const int64_t out = a.first_out + k;
        double X[3], nX[3], px, py;
        child_geometry(sc, rec, a, job, out, X, nX, &px, &py);
        child_write(sc, rec, a, job, out, X, nX, px, py);
    }
}

// ... and, after the tiled photo test of the children, the accept test
__global__ void k_expand_accept(RecordsDev rec, const ExpandArgs a) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const ChildJob job = a.jobs[k];
        const int64_t out = a.first_out + k;
        const double X[3] = {rec.c[3 * out], rec.c[3 * out + 1], rec.c[3 * out + 2]};
        const double nX[3] = {rec.n[3 * out], rec.n[3 * out + 1], rec.n[3 * out + 2]};
        rec.accept[out] = child_accept(rec, a, job.parent, X, nX, rec.count[out]);
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

// Sharded sweep, ingest side: every rank computed the whole sweep's child
// geometry (k_expand_geom) and received the other ranks' photo-test masks,
// so a child's count (|V| = popcount of its mask, MVS2.py:72-74) and its
// accept test (MVS2.py:369) follow here.
__global__ void k_expand_ingest(RecordsDev rec, const ExpandArgs a, int words) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const ChildJob job = a.jobs[k];
        const int64_t out = a.first_out + k;
        int cnt = 0;
        for (int q = 0; q < words; ++q) cnt += __popcll(rec.mask[out * words + q]);
        rec.count[out] = cnt;
        const double X[3] = {rec.c[3 * out], rec.c[3 * out + 1], rec.c[3 * out + 2]};
        const double nX[3] = {rec.n[3 * out], rec.n[3 * out + 1], rec.n[3 * out + 2]};
        rec.accept[out] = child_accept(rec, a, job.parent, X, nX, cnt);
    }
}

// ---------------------------------------------------------------------------
// The multi-GPU sweep's exchange record set (parallel.PointsExchange): the
// accepted candidates of a rank's slice (|V| >= vlb, MVS2.py:256/369) as rows
// [global index, mask words..., (c) x, y, z as binary64 bits] of a
// fixed-capacity buffer whose row 0 is the header [accepted, n, 0...].  No
// host synchronisation: the accepted total travels in the header, and a slice
// with more than cap accepted candidates keeps cap of them (the receiver sees
// accepted > cap).
// One workgroup per chunk of kAccChunk = 8,192 candidates (thread t holds
// candidates chunk + t + 1024 j, j < kAccPer: coalesced loads).  A chunk's
// rows are its accepted candidates in index order; the chunks reserve their
// row ranges by one returning atomic each on the pack's counter, in whatever
// order they get there -- no chunk waits for another (round 5's decoupled
// look-back kept the rows in index order across chunks and cost ~18 us per
// 2^20 sweep); the receiver orders rows by their index column if it needs
// to (PointsExchange.result).  The workgroup that takes the last ticket
// writes the header and returns the counter and the ticket to zero for the
// next call.
// ---------------------------------------------------------------------------
constexpr int kAccThreads = 1024, kAccPer = MVS_ACC_PER, kAccChunk = kAccThreads * kAccPer, kAccWaves = kAccThreads / 64;
constexpr int kAccE = kAccPer * kAccWaves;          // (j, wave) counts of a chunk
constexpr int kAccEpl = (kAccE + 63) / 64;          // of them per lane of wave 0's scan
// 16-B accesses at 8-B alignment (global_load/store_dwordx4 allow it)
typedef double acc_d2v __attribute__((ext_vector_type(2)));
typedef acc_d2v acc_d2 __attribute__((aligned(8)));
typedef long long acc_l2v __attribute__((ext_vector_type(2)));
typedef acc_l2v acc_l2 __attribute__((aligned(8)));
static_assert(kAccChunk == MVS_ACC_CHUNK, "the host sizes the pack's grid by MVS_ACC_CHUNK");
static_assert(kAccE <= 128, "wave 0 scans at most two (j, wave) counts per lane");

// a chunk's ticket, taken after its reservation (base) has returned; the last
// one writes the header and returns the counter and the ticket to zero
DEV void acc_ticket(unsigned long long* __restrict__ ctl, unsigned long long base, int64_t nch, int64_t n, int width,
                    int64_t* __restrict__ out) {
    // the ticket's address depends on the reservation's result (always 0 +
    // 16; opaque to the compiler), so it issues after the return
    const int dep = opaque((int)(base >> 63));
    const unsigned long long tk = atomicAdd(&ctl[16 + dep], 1ull);
    if ((int64_t)tk == nch - 1) {
        const int64_t total = (int64_t)__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[0] = total;
        out[1] = n;
        for (int q = 2; q < width; ++q) out[q] = 0;
        __hip_atomic_store(&ctl[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctl[16], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ctl: [0] the row counter, [16] the chunk ticket (128 B apart), both zero
// between calls
__global__ __launch_bounds__(kAccThreads) void k_acc_pack(int64_t n, int64_t offset, const int32_t* __restrict__ count,
                                                          const uint64_t* __restrict__ mask, const double* __restrict__ cpt,
                                                          int words, int vlb, int64_t cap,
                                                          unsigned long long* __restrict__ ctl,
                                                          int64_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) int32_t s_cnt[kAccE];   // accepted per (j, wave), then their exclusive prefix
    __shared__ int64_t s_base;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int width = 1 + words + (cpt ? 3 : 0);
    // count == null: the scorer's records [mask words, avg], |V| = popcount
    const int64_t ms = count ? words : words + 1;
    const int64_t nch = max((n + kAccChunk - 1) / kAccChunk, (int64_t)1);   // an empty slice still writes the header
    const int64_t b = blockIdx.x;
    // every load of the chunk in flight at once: the first mask words and the
    // counts (records: popcounts of the words)
    uint64_t m[kAccPer], w0[kAccPer];
    int c[kAccPer];
    double px[kAccPer], py[kAccPer], pz[kAccPer];
#pragma unroll
    for (int j = 0; j < kAccPer; ++j) {
        const int64_t i = b * kAccChunk + j * kAccThreads + threadIdx.x;
        w0[j] = i < n ? mask[i * ms] : 0ull;
        c[j] = i < n && count ? count[i] : 0;
    }
#pragma unroll
    for (int j = 0; j < kAccPer; ++j) {
        const int64_t i = b * kAccChunk + j * kAccThreads + threadIdx.x;
        if (i < n && !count) {
            c[j] = __popcll(w0[j]);
            for (int q = 1; q < words; ++q) c[j] += __popcll(mask[i * ms + q]);
        }
    }
    // the accepted candidates' points, in flight across the scan and the
    // reservation (LDS-only barriers)
#pragma unroll
    for (int j = 0; j < kAccPer; ++j) {
        const int64_t i = b * kAccChunk + j * kAccThreads + threadIdx.x;
        const bool acc = i < n && c[j] >= vlb;
        m[j] = __ballot(acc);
        px[j] = py[j] = pz[j] = 0.0;
        if (cpt && acc) {
            // (every candidate's point loaded with the mask words instead --
            // coalesced, but 25 MB instead of the accepted ones' 6 MB:
            // 12.26 vs 11.18 us, profiles/r06/r6u_*)
            // x, y as one 16-B load (8-B aligned), z beside it
            const acc_d2 xy = *(const acc_d2*)(cpt + 3 * i);
            px[j] = xy.x;
            py[j] = xy.y;
            pz[j] = cpt[3 * i + 2];
        }
        if (lane == 0) s_cnt[j * kAccWaves + wave] = __popcll(m[j]);
    }
    lds_barrier();
    if (wave == 0) {
        // exclusive scan of the (j, wave) counts in index order, kAccEpl
        // consecutive ones per lane
        int x[kAccEpl], tot = 0;
#pragma unroll
        for (int q = 0; q < kAccEpl; ++q) {
            const int e = lane * kAccEpl + q;
            x[q] = e < kAccE ? s_cnt[e] : 0;
            tot += x[q];
        }
        int incl = tot;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        int ex = incl - tot;
#pragma unroll
        for (int q = 0; q < kAccEpl; ++q) {
            const int e = lane * kAccEpl + q;
            if (e < kAccE) s_cnt[e] = ex;
            ex += x[q];
        }
        const unsigned long long T = (unsigned)__shfl(incl, 63, 64);   // this chunk's accepted
        if (lane == 0) {
            // this chunk's rows, then its ticket (after the reservation has
            // returned: the last ticket sees every chunk's rows counted)
            const unsigned long long base = T ? atomicAdd(&ctl[0], T) : 0ull;
            s_base = (int64_t)base;
        }
    }
    lds_barrier();
    const int64_t base = s_base;
    // the ticket is taken here, off the rows' critical path (11.07 vs 11.43
    // us with the ticket before the barrier, profiles/r06/r6m_*)
    if (threadIdx.x == 0) acc_ticket(ctl, (unsigned long long)base, nch, n, width, out);
#pragma unroll
    for (int j = 0; j < kAccPer; ++j) {
        if ((m[j] >> lane) & 1ull) {
            const int64_t i = b * kAccChunk + j * kAccThreads + threadIdx.x;
            const int64_t pos = base + s_cnt[j * kAccWaves + wave] +
                                __builtin_amdgcn_mbcnt_hi((uint32_t)(m[j] >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m[j], 0u));
            if (pos < cap && words == 1 && cpt) {
                // the 40-B row as 16 + 16 + 8 B (8-B aligned stores)
                int64_t* o = out + (1 + pos) * width;
                *(acc_l2*)o = acc_l2{offset + i, (int64_t)w0[j]};
                *(acc_l2*)(o + 2) = acc_l2{__double_as_longlong(px[j]), __double_as_longlong(py[j])};
                o[4] = __double_as_longlong(pz[j]);
            } else if (pos < cap) {
                int64_t* o = out + (1 + pos) * width;
                o[0] = offset + i;
                o[1] = (int64_t)w0[j];
                for (int q = 1; q < words; ++q) o[1 + q] = (int64_t)mask[i * ms + q];
                if (cpt) {
                    // the accepted 3D point itself (binary64 bits)
                    o[1 + words] = __double_as_longlong(px[j]);
                    o[2 + words] = __double_as_longlong(py[j]);
                    o[3 + words] = __double_as_longlong(pz[j]);
                }
            }
        }
    }
}

// Measurement only (bench.py exchange.overlap_proxy): a copy of n 16-B pieces
// by a fixed number of workgroups -- the footprint of an RCCL all-gather's
// kernel (a few CUs streaming bytes) -- to run beside the scoring kernels.
// Eight pieces per thread in flight, as a collective's copy loop keeps them
// (one at a time makes the copy latency-bound: 3x slower beside the scorer,
// profiles/r05/r5a_overlap_probe_timeline_old_proxy.txt).
__global__ __launch_bounds__(256) void k_proxy_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
    constexpr int U = 8;
    // one contiguous range per workgroup, U coalesced 4-KiB pieces in flight
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
    for (int64_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + 256 * u < b1 ? src[i + 256 * u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + 256 * u < b1) dst[i + 256 * u] = v[u];
    }
}

// reconstruct_from_Q (MVS2.py:159-173): an accepted patch is appended under
// key (u, cell) for every view u of its V list, with one cell for all entries
// (every V entry carries the projection into the patch's own view), so its
// first sight in the lexicographic key walk is (min u, cell)
__global__ void k_event_keys(RecordsDev rec, int words, const int32_t* __restrict__ events, int64_t n,
                             int nci, int ncj, uint64_t* __restrict__ keys) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = events[e];
        int minv = -1;
        for (int w = 0; w < words && minv < 0; ++w) {
            const uint64_t mk = rec.mask[r * words + w];
            if (mk) minv = 64 * w + __ffsll((long long)mk) - 1;
        }
        const int cx = rec.cell[2 * r], cy = rec.cell[2 * r + 1];
        keys[e] = (minv < 0 || cx < 0 || cx >= nci || cy < 0 || cy >= ncj)
                      ? ~0ull
                      : (uint64_t)(((int64_t)minv * nci + cx) * ncj + cy);
    }
}

// the PLY rows [x y z r g b] (utils.py:249-250) of records idx[i]
__global__ void k_gather_rows(RecordsDev rec, const int32_t* __restrict__ idx, int64_t n,
                              double* __restrict__ rows) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx[i];
        double* o = rows + 6 * i;
        o[0] = rec.c[3 * r];
        o[1] = rec.c[3 * r + 1];
        o[2] = rec.c[3 * r + 2];
        o[3] = rec.color[4 * r];
        o[4] = rec.color[4 * r + 1];
        o[5] = rec.color[4 * r + 2];
    }
}

// avg_ncc_score of accepted patches in the reference's own arithmetic
// (MVS2.py:62-76, for filter_out_outlier): every view of the V list in view
// order, ctNcc in numpy's order (exact_ncc_stack), summed left to right from
// 0 (`self.avg_ncc_score += ncc_score`), then divided by |V|.  One wave per
// record: the lanes score the views, lane 0 sums them in order.  ids == null:
// records 0..n-1 (a scored batch's ref / xy / mask arrays as the records).
template <int WID, int NS>
__global__ __launch_bounds__(256) void k_exact_avg(const SceneDev sc, const RecordsDev rec,
                                                   const int32_t* __restrict__ ids, int64_t n,
                                                   double* __restrict__ out) {
    __shared__ double s_ncc[4][64 * NS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t k = (int64_t)blockIdx.x * 4 + w;
    if (k >= n) return;   // uniform per wave; no block-level barrier below
    const int64_t r = ids ? ids[k] : k;
    const int words = (sc.V + 63) >> 6;
    const int R = rec.R[r];
    int q = 0, rr = 0;
    // a window outside the image has no passing views (its V list is empty);
    // masked views of such a record read a defined NaN, never the stack
    const bool ok = window_ok(sc, rec.xy[2 * r], rec.xy[2 * r + 1], WID, &q, &rr);
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
        const int v = lane + 64 * sl;
        if (v < sc.V && ((rec.mask[r * words + (v >> 6)] >> (v & 63)) & 1ull))
            s_ncc[w][v] = ok ? exact_ncc_stack<WID>(sc, R, v, q, rr) : __builtin_nan("");
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        double sum = 0.0;
        int cnt = 0;
        for (int v = 0; v < sc.V; ++v)
            if ((rec.mask[r * words + (v >> 6)] >> (v & 63)) & 1ull) {
                sum = sum + s_ncc[w][v];
                ++cnt;
            }
        out[k] = cnt ? sum / (double)cnt : 0.0;
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
int launch_score_w(const SceneDev* sc, const ScoreArgs* a, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
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

// hipFuncAttributeMaxDynamicSharedMemorySize of a kernel, set once per device
// (a per-device bit per kernel; racing first launches from two threads may
// both set it, which is harmless)
inline int set_dyn_lds_once(const void* f, std::atomic<uint64_t>& done, int lds) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    const uint64_t bit = dev < 64 ? (1ull << dev) : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return 0;
    if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return -1;
    done.fetch_or(bit, std::memory_order_release);
    return 0;
}

template <int WID, int NBLK, bool GROUPED>
int launch_mma(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, const MomentsDev* mt, hipStream_t s) {
    static std::atomic<uint64_t> attr_fast{0}, attr_slow{0}, attr_fast2{0}, attr_slow2{0};
    if constexpr (GROUPED) {
        // (mt: the scene's S_b / D tables, or null: the Q table per item and group)
        const MomentsDev m0{};
        const MomentsDev& m = mt ? *mt : m0;
        if (mt) {
            constexpr int lds = v_lds<true>().total;
            if (fabs(a->thr) >= 0.01) {
                if (set_dyn_lds_once((const void*)k_score_mma_v<WID, true, true>, attr_fast, lds) != 0) return -1;
                hipLaunchKernelGGL((k_score_mma_v<WID, true, true>), dim3(kMmaGrid), dim3(kMmaThreads), lds, s, *sc,
                                   *a, *t, m, (const int4*)t->items, (const int2*)t->sorted);
            } else {
                if (set_dyn_lds_once((const void*)k_score_mma_v<WID, false, true>, attr_slow, lds) != 0) return -1;
                hipLaunchKernelGGL((k_score_mma_v<WID, false, true>), dim3(kMmaGrid), dim3(kMmaThreads), lds, s, *sc,
                                   *a, *t, m, (const int4*)t->items, (const int2*)t->sorted);
            }
        } else {
            constexpr int lds = v_lds<false>().total;
            if (fabs(a->thr) >= 0.01) {
                if (set_dyn_lds_once((const void*)k_score_mma_v<WID, true, false>, attr_fast2, lds) != 0) return -1;
                hipLaunchKernelGGL((k_score_mma_v<WID, true, false>), dim3(kMmaGrid), dim3(kMmaThreads), lds, s, *sc,
                                   *a, *t, m, (const int4*)t->items, (const int2*)t->sorted);
            } else {
                if (set_dyn_lds_once((const void*)k_score_mma_v<WID, false, false>, attr_slow2, lds) != 0) return -1;
                hipLaunchKernelGGL((k_score_mma_v<WID, false, false>), dim3(kMmaGrid), dim3(kMmaThreads), lds, s, *sc,
                                   *a, *t, m, (const int4*)t->items, (const int2*)t->sorted);
            }
        }
    } else {
        // the largest table is sized for V = 16 NBLK; every V of this NBLK fits in it
        const int lds = mma_layout<WID, NBLK>(16 * NBLK).total;
        const int used = mma_layout<WID, NBLK>(sc->V).total;
        if (fabs(a->thr) >= 0.01) {
            if (set_dyn_lds_once((const void*)k_score_mma<WID, NBLK, true>, attr_fast, lds) != 0) return -1;
            hipLaunchKernelGGL((k_score_mma<WID, NBLK, true>), dim3(kMmaGrid), dim3(kMmaThreads), used, s, *sc, *a,
                               *t, (const int4*)t->items, (const int2*)t->sorted);
        } else {
            if (set_dyn_lds_once((const void*)k_score_mma<WID, NBLK, false>, attr_slow, lds) != 0) return -1;
            hipLaunchKernelGGL((k_score_mma<WID, NBLK, false>), dim3(kMmaGrid), dim3(kMmaThreads), used, s, *sc,
                               *a, *t, (const int4*)t->items, (const int2*)t->sorted);
        }
    }
    return 0;
}

template <int WID>
int launch_score_tiled_w(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, const MomentsDev* mt,
                         hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    if (a->n == 0) return 0;
    const bool grouped = sc->V > kGroupViews;
    if (t->tw != MVS_TILE_W || t->th != MVS_TILE_H || t->items == nullptr ||
        t->chunk != (grouped ? kGroupChunk : kMmaChunk) || t->groups != (grouped ? (sc->V + 63) / 64 : 1) ||
        sc->V > MVS_MAX_VIEWS)
        return -3;
    // tile counters and the control block (queue heads, fix_count, n_items)
    // of this parity: zeroed by the previous batch's k_bin, unless
    // zero_first (both sets)
    if (t->zero_first &&
        (hipMemsetAsync(t->tile_count, 0, sizeof(int32_t) * tc_words(t->ntiles), s) != hipSuccess ||
         hipMemsetAsync(t->zero_blk, 0, sizeof(int32_t) * t->zero_words, s) != hipSuccess))
        return -1;
    const int64_t per_block = (int64_t)kBinBlock * kBinPer;
    const int nbin = (int)((a->n + per_block - 1) / per_block);
    // k_score_tab on a dense batch (>= kImplicitMean candidates per tile on
    // average: every tile holds some, so an empty item is rare) takes the
    // tiles themselves as its items, in tile order, and needs no k_item_scan
    TiledArgs tv = *t;
    tv.implicit = (!grouped && mt && a->n >= (int64_t)kImplicitMean * t->ntiles) ? 1 : 0;
    // with the scene's moment tables k_bin also settles the candidates whose
    // reference window is constant (they pass no view) without binning them
    const MomentsDev mflat = mt ? *mt : MomentsDev{};
    if (t->ntiles <= kBinLdsTiles)
        hipLaunchKernelGGL(k_bin<true>, dim3(nbin), dim3(kBinBlock), (size_t)t->ntiles * 4, s, *sc, *a, tv, WID, mflat);
    else
        hipLaunchKernelGGL(k_bin<false>, dim3(nbin), dim3(kBinBlock), 0, s, *sc, *a, tv, WID, mflat);
    // the work items in tile order (the scorers' workgroups in flight then
    // share image rows -- and at V > 64 table rows -- in L2)
    if (!tv.implicit) hipLaunchKernelGGL(k_item_scan, dim3(1), dim3(kScanThreads), 0, s, tv);
    t = &tv;
    int rc = 0;
    {
        TimedLaunch tl(s, ev0, ev1);
        if (grouped) rc = launch_mma<WID, 4, true>(sc, a, t, mt, s);
        else if (mt) rc = mvs_launch_score_tab(sc, a, t, mt, s);   // window moments from the scene's tables
        else switch ((sc->V + 15) / 16) {
            case 1: rc = launch_mma<WID, 1, false>(sc, a, t, nullptr, s); break;
            case 2: rc = launch_mma<WID, 2, false>(sc, a, t, nullptr, s); break;
            case 3: rc = launch_mma<WID, 3, false>(sc, a, t, nullptr, s); break;
            default: rc = launch_mma<WID, 4, false>(sc, a, t, nullptr, s); break;
        }
    }
    if (rc) return rc;
    // 256 waves (one candidate each at a time) for the guard band; up to 4x as
    // many for a batch whose overflow list is long
    const int kFixBlocks = (int)std::min<int64_t>(std::max<int64_t>(a->n / 4096, kFixBase), 4 * kFixBase);
    if (grouped) {
        if (sc->V <= 128)
            hipLaunchKernelGGL((k_score_fix<WID, 2>), dim3(kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
        else
            hipLaunchKernelGGL((k_score_fix<WID, 4>), dim3(kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
    } else {
        hipLaunchKernelGGL((k_score_fix<WID, 1>), dim3(kFixBlocks), dim3(256), 0, s, *sc, *a, *t);
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

int grid_for(int64_t n, int block, int cap) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + block - 1) / block, cap));
}

}  // namespace

#ifdef MVS_STAMPS
extern "C" int mvs_read_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int mvs_launch_build_scene(const SceneDev* sc, const uint8_t* d_rgb, uint8_t* d_stack,
                                      uint8_t* d_gv_base, hipStream_t s) {
    (void)d_gv_base;
    const dim3 grid((unsigned)((sc->W + kSceneStrip - 1) / kSceneStrip), (unsigned)sc->H);
    hipLaunchKernelGGL(k_build_scene, grid, dim3(256), 0, s, *sc, d_rgb, d_stack, (uint8_t*)sc->gv);
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

template <int WID>
size_t mma_lds_bytes_w(int V) {
    if (V > kGroupViews) return (size_t)(v_lds<false>().total + v_static_lds<WID>());
    switch ((V + 15) / 16) {
        case 1: return (size_t)mma_layout<WID, 1>(V).total;
        case 2: return (size_t)mma_layout<WID, 2>(V).total;
        case 3: return (size_t)mma_layout<WID, 3>(V).total;
        default: return (size_t)mma_layout<WID, 4>(V).total;
    }
}

extern "C" size_t mvs_mma_lds_bytes(int V, int wid) {
    switch (wid) {
        case 1: return mma_lds_bytes_w<1>(V);
        case 2: return mma_lds_bytes_w<2>(V);
        case 3: return mma_lds_bytes_w<3>(V);
        case 4: return mma_lds_bytes_w<4>(V);
        case 5: return mma_lds_bytes_w<5>(V);
        default: return 0;
    }
}

extern "C" const char* mvs_timed_kernel_name(int V, int wid, int tiled) {
    (void)wid;
    if (!tiled) return "k_score";
    if (tiled == 2) return "k_score_tab";
    return V > kGroupViews ? "k_score_mma_v" : "k_score_mma";
}

extern "C" int mvs_launch_score_tiled(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, int wid,
                                      const MomentsDev* mt, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    switch (wid) {
        case 1: return launch_score_tiled_w<1>(sc, a, t, mt, s, ev0, ev1);
        case 2: return launch_score_tiled_w<2>(sc, a, t, mt, s, ev0, ev1);
        case 3: return launch_score_tiled_w<3>(sc, a, t, mt, s, ev0, ev1);
        case 4: return launch_score_tiled_w<4>(sc, a, t, mt, s, ev0, ev1);
        case 5: return launch_score_tiled_w<5>(sc, a, t, mt, s, ev0, ev1);
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

extern "C" int mvs_launch_expand_geom(const SceneDev* sc, RecordsDev rec, const ExpandArgs* a, hipStream_t s) {
    if (a->n <= 0) return 0;
    hipLaunchKernelGGL(k_expand_geom, dim3(grid_for(a->n, 256, 4096)), dim3(256), 0, s, *sc, rec, *a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_expand_accept(RecordsDev rec, const ExpandArgs* a, hipStream_t s) {
    if (a->n <= 0) return 0;
    hipLaunchKernelGGL(k_expand_accept, dim3(grid_for(a->n, 256, 4096)), dim3(256), 0, s, rec, *a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_pack_accepted(int64_t n, int64_t offset, const int32_t* count, const uint64_t* mask,
                                        const double* c, int words, int vlb, int64_t cap, unsigned long long* ctl,
                                        int64_t* out, hipStream_t s) {
    const int64_t nchunk = (n + kAccChunk - 1) / kAccChunk;
    if (nchunk >= ((int64_t)1 << 31)) return -3;
    const int grid = (int)std::max<int64_t>(1, nchunk);   // one workgroup per chunk
    // n == 0 still writes the header (chunk 0 of an empty slice)
    hipLaunchKernelGGL(k_acc_pack, dim3(grid), dim3(kAccThreads), 0, s, n, offset, count, mask, c, words, vlb, cap,
                       ctl, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_proxy_copy(void* dst, const void* src, int64_t bytes, int workgroups, hipStream_t s) {
    if (bytes <= 0) return 0;
    hipLaunchKernelGGL(k_proxy_copy, dim3(std::max(workgroups, 1)), dim3(256), 0, s, (const uint4*)src, (uint4*)dst,
                       bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_expand_ingest(RecordsDev rec, const ExpandArgs* a, int words, hipStream_t s) {
    if (a->n <= 0) return 0;
    hipLaunchKernelGGL(k_expand_ingest, dim3(grid_for(a->n, 256, 4096)), dim3(256), 0, s, rec, *a, words);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int mvs_launch_ncc_windows(int64_t n, int npx, const uint8_t* a, const uint8_t* b,
                                      double thr, int force_exact, double* ncc, uint8_t* pass,
                                      hipStream_t s) {
    if (npx <= 0 || npx > 128) return -2;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_ncc_windows, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, n, npx, a, b, thr,
                       force_exact, ncc, pass);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_event_keys(RecordsDev rec, int words, const int32_t* events, int64_t n_events,
                                     int nci, int ncj, uint64_t* keys, hipStream_t s) {
    if (n_events <= 0) return 0;
    hipLaunchKernelGGL(k_event_keys, dim3(grid_for(n_events, 256, 4096)), dim3(256), 0, s, rec, words, events,
                       n_events, nci, ncj, keys);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int WID>
int launch_exact_avg_w(const SceneDev* sc, RecordsDev rec, const int32_t* ids, int64_t n, double* out,
                       hipStream_t s) {
    const dim3 grid((unsigned)((n + 3) / 4));
    if (sc->V <= 64) hipLaunchKernelGGL((k_exact_avg<WID, 1>), grid, dim3(256), 0, s, *sc, rec, ids, n, out);
    else if (sc->V <= 128) hipLaunchKernelGGL((k_exact_avg<WID, 2>), grid, dim3(256), 0, s, *sc, rec, ids, n, out);
    else hipLaunchKernelGGL((k_exact_avg<WID, 4>), grid, dim3(256), 0, s, *sc, rec, ids, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_exact_avg(const SceneDev* sc, RecordsDev rec, int wid, const int32_t* ids, int64_t n,
                                    double* out, hipStream_t s) {
    if (n <= 0) return 0;
    if (sc->V > MVS_MAX_VIEWS) return -3;
    switch (wid) {
        case 3: return launch_exact_avg_w<3>(sc, rec, ids, n, out, s);
        case 5: return launch_exact_avg_w<5>(sc, rec, ids, n, out, s);
        default: return -2;
    }
}

extern "C" int mvs_launch_gather_rows(RecordsDev rec, const int32_t* idx, int64_t n, double* rows, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_gather_rows, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, rec, idx, n, rows);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Stable sort of (key, value) pairs on the device (hipCUB LSD radix sort over
// the low `bits` key bits); tmp / tmp_bytes as hipcub: call with tmp == NULL
// to size the scratch.
extern "C" int mvs_sort_pairs(void* tmp, size_t* tmp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                              const int32_t* vals_in, int32_t* vals_out, int64_t n, int bits, hipStream_t s) {
    if (hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0, bits,
                                           s) != hipSuccess)
        return -1;
    return 0;
}

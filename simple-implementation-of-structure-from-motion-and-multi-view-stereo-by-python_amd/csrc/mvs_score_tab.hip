// The tiled matrix-core photo test for V <= 64 with per-scene window moments
// (gfx950 / CDNA4).
//
// Reference path: MyPatch.photo_consistenecy_test (MVS2.py:62-77) -> ctNcc
// (MVS2.py:39-43) of every view's window (getDescFeatures,
// HarrisFeatures.py:116-133) against the reference view's, all at the
// reference view's pixel (MVS2.py:68).
//
// ctNcc(a, b) = n (n S_ab - S_a S_b) / ((n-1) sqrt(D_a) sqrt(D_b)),
// D = n S_xx - S_x^2.  Everything but S_ab depends on one (pixel, view)
// window alone, and the scene is immutable: k_moments computes S_b and
// w_b = 1/sqrt(D_b) once per scene (and window size) into two pixel-major
// tables, and the scorer k_score_tab only forms the window products S_ab on
// the matrix cores (v_mfma_i32_16x16x64_i8 over the tile's staged region, as
// k_score_mma does) and takes the decision num w_b > T from the tables.
#include <algorithm>

#include "mvs_device.h"
#include "mvs_mma.h"

namespace {

// ---------------------------------------------------------------------------
// k_moments: S_b and w_b of every (pixel, view) with a valid window
// (getDescFeatures' bounds, HarrisFeatures.py:128), 32 columns x 16 rows x 16
// views per workgroup.  The gray bytes of the block's views and rows land in
// LDS; per (view, column) a thread forms every row's horizontal window sums
// (S = sum g, Q = sum g^2 of the unsigned g, packed Q << 12 | S) by byte dot
// products in registers, and the vertical sums slide down the 16 rows.  The same arithmetic as the
// in-kernel moments of k_score_mma (the tables are bit-identical to them):
// D = n Q - S^2 (exact int32), w = v_rsq_f64(D) + one Newton step (a constant
// window: D = 0, inf, then nan), S_b = S - 128 n; and a bit per (pixel, view)
// for D = 0.  Stores: lanes = 16 views x 4 pixels, one 128-B row piece of w
// per pixel.
// ---------------------------------------------------------------------------
constexpr int kMomW = 32, kMomH = 16, kMomV = 16;

template <int WID, bool DTAB>
__global__ __launch_bounds__(256) void k_moments(const SceneDev sc, const MomentsDev mt) {
    constexpr int NB = 2 * WID + 1, NPX = NB * NB;
    // LDS column c holds image column x0 - 8 + c: 48 bytes cover the block's
    // 32 columns and both window halos (WID <= 5 < 8); rows of 13 dwords
    // (the lanes of a read are 16 views x 4 columns: a view stride of 13 ROWS
    // dwords spreads them over the banks).  The only LDS array: 21 KB at
    // WID 5, so up to 7 workgroups share a CU (a 58 KB table of the
    // horizontal sums held it to 2: 73 us per dinoRing scene)
    constexpr int ROWS = kMomH + 2 * WID, CP = 48, CW = CP / 4, GP = CW + 1;
    __shared__ __attribute__((aligned(16))) uint32_t g4[kMomV][ROWS][GP];
    const int x0 = blockIdx.x * kMomW, y0 = blockIdx.y * kMomH, v0 = blockIdx.z * kMomV;
    const int tid = threadIdx.x;
    const int nv = min(kMomV, sc.V - v0);
    // the bytes, one dword per thread and step, coalesced along each row: gv
    // rows (signed s = g - 128; 8 pad bytes left of column 0 and >= 24 right
    // of W-1, so [x0 - 8, x0 + 40) is inside the row's pitch or, for the last
    // columns, the next row's start / the buffer's 64-byte tail, never used
    // by a valid window); rows outside the image clamped; views past V zero.
    // Every load of the thread in flight at once, then the LDS writes (a
    // load-then-write loop waited for each load in turn)
    constexpr int NLD = kMomV * ROWS * CW, PER = (NLD + 255) / 256;
    uint32_t buf[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int k = tid + 256 * j;
        const int vi = k / (ROWS * CW), rc = k - vi * (ROWS * CW), r = rc / CW, c = rc - r * CW;
        const int y = min(max(y0 - WID + r, 0), sc.H - 1);
        uint32_t wv = 0u;
        if (k < NLD && vi < nv)
            wv = *(const uint32_t*)(sc.gv + ((int64_t)(v0 + vi) * sc.H + y) * sc.Wp + x0 - 8 + 4 * c);
        buf[j] = wv;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int k = tid + 256 * j;
        const int vi = k / (ROWS * CW), rc = k - vi * (ROWS * CW), r = rc / CW, c = rc - r * CW;
        if (k < NLD) g4[vi][r][c] = vi < nv ? buf[j] ^ 0x80808080u : 0u;
    }
    __syncthreads();
    const int x_lo = WID + 1, x_hi = sc.W - WID - 2, y_lo = WID, y_hi = sc.H - WID - 2;   // valid centres
    // the window's NB bytes of a row: NF whole aligned dwords and NR bytes
    constexpr int NF = NB / 4, NR = NB % 4, ND = NF + (NR ? 1 : 0);
    // a task = (view, column, half of the block's rows): 8 output rows from
    // 8 + 2 WID rows of horizontal sums (fewer live registers than all 16)
    constexpr int OH = kMomH / 2, RH = OH + 2 * WID;
    for (int k = tid; k < kMomV * kMomW * 2; k += 256) {
        const int vi = k & (kMomV - 1), xl = (k >> 4) & (kMomW - 1), rb = (k >> 9) * OH;
        const int x = x0 + xl;
        if (x < x_lo || x > x_hi) continue;
        // per row r of the block: the horizontal window sums S = sum g and
        // Q = sum g^2 of the unsigned bytes (exact integers, packed Q << 12 |
        // S) by byte dot products over the window's bytes, realigned from
        // the row's dwords; every row's reads in flight together
        const int b0 = 8 - WID + xl, sh = b0 & 3, d0 = b0 >> 2;   // image column x - WID
        uint32_t hp[RH];
#pragma unroll
        for (int r = 0; r < RH; ++r) {
            const uint32_t* gr = &g4[vi][rb + r][d0];
            uint32_t wd[ND + 1];
#pragma unroll
            for (int j = 0; j <= ND; ++j) wd[j] = gr[j];
            uint32_t S = 0u, Q = 0u;
#pragma unroll
            for (int j = 0; j < ND; ++j) {
                uint32_t a = __builtin_amdgcn_alignbyte(wd[j + 1], wd[j], (uint32_t)sh);
                if (j == NF) a &= (1u << (8 * NR)) - 1u;
                S = __builtin_amdgcn_udot4(a, 0x01010101u, S, false);
                Q = __builtin_amdgcn_udot4(a, a, Q, false);
            }
            hp[r] = (Q << 12) | S;
        }
        int S = 0, Q = 0;
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            S += (int)(hp[r] & 0xfffu);
            Q += (int)(hp[r] >> 12);
        }
#pragma unroll
        for (int yl = 0; yl < OH; ++yl) {
            if (yl > 0) {
                const uint32_t a = hp[yl - 1], b = hp[yl + NB - 1];
                S += (int)(b & 0xfffu) - (int)(a & 0xfffu);
                Q += (int)(b >> 12) - (int)(a >> 12);
            }
            const int y = y0 + rb + yl;
            if (y < y_lo || y > y_hi) continue;
            const int64_t o = ((int64_t)y * sc.W + x) * mt.VP + v0 + vi;
            // the constant windows (D = 0) of the pixel's 16 views as one
            // 16-bit word: lanes = 16 views x 4 pixels (k_bin's flat test)
            const uint64_t fb = __ballot(vi < nv && NPX * Q - S * S == 0);
            if (mt.flat && vi == 0)
                mt.flat[((int64_t)y * sc.W + x) * (mt.VP / 16) + v0 / 16] =
                    (uint16_t)(fb >> (16 * ((threadIdx.x >> 4) & 3)));
            if (vi < nv) {
                const int db = NPX * Q - S * S;
                mt.sb[o] = (int16_t)(S - 128 * NPX);
                if constexpr (DTAB) {
                    mt.d[o] = db;
                } else {
                    const double D = (double)db;
                    double w = __builtin_amdgcn_rsq(D);
                    w = w * (1.5 - 0.5 * D * w * w);
                    mt.w[o] = w;
                }
            } else {
                mt.sb[o] = 0;
                if constexpr (DTAB) mt.d[o] = -1;
                else {
                    mt.w[o] = __builtin_nan("");
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_score_tab (V <= 64).  Two workgroups of 8 waves per CU (each <= 80 KiB of
// LDS), each taking work items -- the candidates of one 16x8 pixel tile, at
// most kMmaChunk -- from the dynamic queue k_bin's item scan built (tile
// order).  Per item:
//   1. the item's window region of every view (signed bytes, [view][ROWS][32],
//      one pad row per view) and its candidate list are in LDS (LDS-DMA,
//      double-buffered where LDS allows: item k+1's lands while item k is
//      scored; a barrier per item);
//   2. wave w takes the item's M-blocks [w nblk / 8, (w+1) nblk / 8) and sorts
//      its own candidates by row pair (ballots, in its own part of the list:
//      no workgroup barrier), so that a unit's windows span few K-steps;
//   3. units of two M-blocks of 16 candidates: C[m][v] = sum over the window
//      of s_R s_v by v_mfma_i32_16x16x64_i8 (A = the reference window masked
//      to candidate m's window, B = view v's region), exact; meanwhile S_b,
//      w_b of the unit's pixels come from the tables (global loads, one
//      candidate step ahead of their use);
//   4. num = n C - S_a S_b, ncc > thr <=> num w_b > T = thr (n-1)/(n w_a): one
//      binary32 fma per (candidate, view), guard band 2e-6 |T| (k_score_fix
//      re-scores a candidate with a pair inside it), the passing terms
//      summed in binary64 (avg_ncc_score).
// The other workgroup on the CU fills the issue slots this one leaves at its
// barrier and in its latency waits.
// ---------------------------------------------------------------------------
#ifdef MVS_STAMPS
// diagnostic build only: per-workgroup cycle sums (lane 0 of every wave adds
// its own): slot 0 rounds (wave 0), 1 barrier wait at the round's start, 2
// the wave's sort (from the barrier: incl. 7), 3 its units, 4 its M-blocks,
// 5 K-loops, 6 epilogues, 7 the next item's LDS-DMA issue and loads;
// read by mvs_read_stamps_tab
__device__ unsigned long long g_stamps_tab[1024 * 16];
#define TSTAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define TSTAMP_ADD(slot, val) \
    do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_stamps_tab[(blockIdx.x & 1023) * 16 + (slot)], (unsigned long long)(val)); } while (0)
#else
#define TSTAMP(var)
#define TSTAMP_ADD(slot, val)
#endif

// The A/B variants measured against this kernel in rounds 4-5 (split and
// transposed epilogues, binary64 decisions, pixel sorts, LDS table rows, DMA
// issue by fewer waves or later, 10 waves, tail-split items, one workgroup
// per CU, ...) are in DESIGN.md 4.1 with their logs under profiles/r05/; the
// code of each is in the git history (round 5), not in this file.
constexpr int kTabWaves = 8, kTabThreads = 64 * kTabWaves, kTabGrid = 512;
constexpr int kTabBudget = 80 * 1024 - 512;                 // LDS bytes per workgroup (two per CU)
constexpr int kTabMinWaves = (2 * kTabWaves + 3) / 4;       // per SIMD
constexpr int kTabChunk = MVS_MMA_CHUNK;

// a candidate's constants in a unit (per wave, 32 slots)
struct alignas(16) TabInfo {
    int32_t tix;   // table element of its pixel, view 0
    int32_t Sa;    // -S_a
    int32_t R;     // reference view (-1: no candidate)
    float T;       // decision threshold on num w_b (FAST)
};

template <int WID, int NBLK>
struct TabGeom {
    static constexpr int VP = 16 * NBLK;
    static constexpr int RB = VP * MmaGeom<WID>::VS;    // one region buffer (+16 zero bytes)
    static constexpr int CB = kTabChunk * 8;            // one candidate buffer
    static constexpr int FIXED = kTabWaves * 32 * (int)sizeof(TabInfo) + 65 * 8 + 64;
    static constexpr int BUF = (RB + 16) + CB;          // one item's LDS
    static_assert(BUF + FIXED <= kTabBudget, "one item's buffers fit");
    // two buffer sets where they fit: item k+1's lands while item k is scored
    static constexpr bool DB = 2 * BUF + FIXED <= kTabBudget;
};

template <int WID, int NBLK, bool FAST>
__global__ __launch_bounds__(kTabThreads, kTabMinWaves) void k_score_tab(const SceneDev sc, const ScoreArgs a, const TiledArgs t,
                                                               const MomentsDev mt, const int4* __restrict__ items,
                                                               const int2* __restrict__ sorted) {
    using G = MmaGeom<WID>;
    using TG = TabGeom<WID, NBLK>;
    constexpr int NB = G::NB, NPX = G::NPX, KS = G::KS, VS = G::VS, C0 = G::C0;
    constexpr int VP = TG::VP;
    constexpr bool DB = TG::DB;

    constexpr int RPV = VS / 32;                                          // region rows per view incl. the pad row
    constexpr int PF = (VP * RPV * 2 + kTabThreads - 1) / kTabThreads;    // 16-B pieces per thread
    constexpr int RB = TG::RB, CB = TG::CB;
    // distinct LDS objects per buffer: reads of one do not wait for the
    // LDS-DMA into the other; each region buffer ends in 16 zero bytes (rows
    // outside a window read them by an offset select inside the same buffer)
    __shared__ __attribute__((aligned(16))) uint8_t s_reg0[RB + 16], s_reg1[DB ? RB + 16 : 16];
    __shared__ __attribute__((aligned(16))) uint8_t s_cand0[CB], s_cand1[DB ? CB : 16];
    __shared__ __attribute__((aligned(16))) TabInfo s_ti[kTabWaves * 32];
    __shared__ int s_ids[2];
    __shared__ double s_recip[65];
#ifdef MVS_STAMPS
    const unsigned long long t_wg0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int V = sc.V;
    const int npiece = V * RPV * 2;
    if (tid <= 64) s_recip[tid] = c_recip.r[tid];
    if (tid < 4) ((uint32_t*)(s_reg0 + RB))[tid] = 0u;
    if (DB && tid >= 4 && tid < 8) ((uint32_t*)(s_reg1 + RB))[tid & 3] = 0u;
    TabInfo* ti = s_ti + wave * 32;

    const double kn = (double)NPX / (double)(NPX - 1);
    const float tqf = (float)(a.thr / kn);
    ItemMap im;
    im.load(t);
    // implicit items: k < ntiles is (tile k, chunk 0), then segment 1's
    // further chunks (k_bin); else k_item_scan's list
    const bool implicit = t.implicit != 0;
    const int n_units = implicit ? t.ntiles + t.n_items[32] : im.total();
    int32_t* head = t.head;
    const int16_t* __restrict__ tsb = mt.sb;
    const double* __restrict__ tw = mt.w;

    auto region_buf = [&](auto bufc) -> uint8_t* { return decltype(bufc)::value ? s_reg1 : s_reg0; };
    auto cand_buf = [&](auto bufc) -> uint8_t* { return decltype(bufc)::value ? s_cand1 : s_cand0; };
    // the item's region (gv rows) and sorted (id, pk) entries by LDS-DMA
    auto stage = [&](const int4 d, auto bufc) {
        const int ty = d.x / t.ntx, tx = d.x - ty * t.ntx;
        const int x0 = tx * MVS_TILE_W, yr0 = ty * MVS_TILE_H - WID;
        uint8_t* base = region_buf(bufc);
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int k = opaque(tid) + p * kTabThreads;   // recomputed per piece: no long-lived offsets
            const int v = k / (2 * RPV), r2 = k - v * (2 * RPV);
            // the pad row (never read) is not loaded (its lanes masked)
            if (k < npiece && (r2 >> 1) != RPV - 1) {
                const int y = min(max(yr0 + (r2 >> 1), 0), sc.H - 1);
                const uint8_t* src = sc.gv + ((int64_t)v * sc.H + y) * sc.Wp + (x0 - 8) + 16 * (r2 & 1);
                __builtin_amdgcn_global_load_lds((const void*)src,
                                                 (void __attribute__((address_space(3)))*)(base + (p * kTabThreads + wave * 64) * 16),
                                                 16, 0, 0);
            }
        }
        // the list in 16-B pieces (two entries; bucket starts are 512-B
        // aligned and d.w even): one DMA instruction per wave for a chunk
        uint8_t* cbase = cand_buf(bufc);
        const uint8_t* csrc = (const uint8_t*)(sorted + d.y);
#pragma unroll
        for (int p = 0; p < (kTabChunk / 2 + kTabThreads - 1) / kTabThreads; ++p) {
            const int k = tid + p * kTabThreads;
            if (k < d.w / 2)
                __builtin_amdgcn_global_load_lds((const void*)(csrc + 16 * k),
                                                 (void __attribute__((address_space(3)))*)(cbase + (p * kTabThreads + wave * 64) * 16),
                                                 16, 0, 0);
        }
    };

    // The items in kBands contiguous bands of tiles, band x served first by
    // the workgroups b = x mod kBands -- one band per XCD under the
    // round-robin dispatch, so that an XCD's workgroups in flight take
    // neighbouring tiles and share their regions' lines in its L2 (76.4 vs
    // 78.9 us with one queue, profiles/r06/r6n_*) -- each band with its own
    // queue head.  A band's first 2 x (its workgroups) items are handed out
    // without a claim (workgroup l of the band takes items l and l + its
    // workgroups: at the kernel's start the grid's claims would otherwise
    // queue on the heads); a workgroup whose band is
    // exhausted claims from the next bands.
    constexpr int kBands = kBandHeads;
    const int ob = (int)blockIdx.x % kBands;
    int32_t* bheads = head + (3 + kItemSegs) * 32;   // band x's head at bheads[32 x]
    auto bstart = [&](int x) -> int { return (int)((int64_t)n_units * x / kBands); };
    auto bwgs = [&](int x) -> int { return ((int)gridDim.x - x + kBands - 1) / kBands; };
    int cb = ob;   // thread 0's: the band it claims from
    auto claim = [&]() -> int {
        return band_claim(bheads, cb, ob, kBands, n_units, [&](int x) { return 2 * bwgs(x); });
    };
    // an item's descriptor (tile, first bucket entry, count, entries staged):
    // the list is staged as a whole chunk (bounded by the bucket), so that its
    // LDS-DMA needs no count -- the count arrives a round later
    auto desc = [&](int2 it, int cnt) -> int4 {
        const int tile = __builtin_amdgcn_readfirstlane(it.x), j = __builtin_amdgcn_readfirstlane(it.y);
        const int c = __builtin_amdgcn_readfirstlane(cnt);
        return make_int4(tile, tile * t.cap + j * t.chunk, min(min(c, t.cap) - j * t.chunk, t.chunk),
                         min(t.chunk, t.cap - j * t.chunk));
    };
    // an item's (tile, chunk): implicit items below ntiles are computed (no
    // load: the round's DMA issue then waits for nothing; the load and the
    // select of round 5 made every wave wait a memory round trip there);
    // else a vector load (a lane-dependent-looking address)
    auto item_v = [&](int v) -> int2 {
        if (implicit && v < t.ntiles) return make_int2(v, 0);
        return *(const int2*)(items + opaque(implicit ? t.item_seg + max(v - t.ntiles, 0) : im.slot(v)));
    };
    auto count_v = [&](int tile) -> int { return t.tile_count[opaque(tile * kTcStride)]; };
    // the item pipeline: while item k is scored, item k+1's region and list
    // (DB) and its tile's count are in flight, and thread 0 claims item k+2
    // after wave 0's first unit of item k (the index goes round through LDS at
    // the next round's barrier)
    if (tid == 0) {
        const int l = (int)blockIdx.x / kBands, bs = bstart(ob), bn = bstart(ob + 1) - bs;
        const int s0 = l < bn ? bs + l : -1, s1 = l + bwgs(ob) < bn ? bs + l + bwgs(ob) : -1;
        const int c0 = s0 >= 0 ? s0 : claim();
        s_ids[0] = c0;
        s_ids[1] = s1 >= 0 ? s1 : c0 < n_units ? claim() : n_units;
    }
    __syncthreads();
    int cur = __builtin_amdgcn_readfirstlane(s_ids[0]);
    int nx1 = __builtin_amdgcn_readfirstlane(s_ids[1]);
    if (cur >= n_units) return;
    int4 dcur;
    {
        // an implicit item needs no load; the first DMA needs no count (its
        // list is staged as a whole chunk), so it goes out before the count
        const int2 it = implicit && cur < t.ntiles ? make_int2(cur, 0) : item_v(cur);
        const int tile = __builtin_amdgcn_readfirstlane(it.x), j = __builtin_amdgcn_readfirstlane(it.y);
        stage(make_int4(tile, tile * t.cap + j * t.chunk, 0, min(t.chunk, t.cap - j * t.chunk)),
              std::integral_constant<int, 0>{});
        dcur = desc(it, count_v(it.x));
    }
    int2 it1 = make_int2(0, 0);
    int pend = nx1;   // thread 0's: the next item, published at round 0's barrier
    __syncthreads();   // everyone has read s_ids before they are rewritten

    auto round = [&](auto bufc) -> bool {
        constexpr int buf = decltype(bufc)::value;
        const int nc = dcur.z;
        const uint8_t* reg = region_buf(bufc);
        int2* cand = (int2*)cand_buf(bufc);
        const int zoff = RB;   // the zero row, relative to the region buffer
        // ---- 1. this item's region and list have landed (every wave's DMA) ----
        TSTAMP(ts0);
        if (tid == 0) s_ids[0] = pend;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's LDS-DMA, before the barrier
        __syncthreads();
        TSTAMP(ts1);
        // item k+1 (claimed last round), its region and list into the other
        // buffer and its count
        nx1 = __builtin_amdgcn_readfirstlane(s_ids[0]);
        if (nx1 < n_units) {
            const int2 iv = item_v(nx1);   // implicit: computed; else a load waited for here
            it1 = make_int2(__builtin_amdgcn_readfirstlane(iv.x), __builtin_amdgcn_readfirstlane(iv.y));
        }
        const int j1 = it1.y;
        const int4 dst1 = make_int4(it1.x, it1.x * t.cap + j1 * t.chunk, 0, min(t.chunk, t.cap - j1 * t.chunk));
        if constexpr (DB) {
            if (nx1 < n_units) stage(dst1, std::integral_constant<int, buf ^ 1>{});
        }
        const int c1 = count_v(it1.x);
        TSTAMP(ts1b);
        TSTAMP_ADD(7, ts1b - ts1);
        const int ty = dcur.x / t.ntx, tx = dcur.x - ty * t.ntx;
        const int tix0 = ((ty * MVS_TILE_H) * sc.W + tx * MVS_TILE_W) * VP;   // table element of the tile origin
        // ---- 2. this wave's M-blocks, sorted by row pair inside the wave ----
        const int nblk = (nc + 15) >> 4;
        const int b0 = nblk * wave / kTabWaves, b1 = nblk * (wave + 1) / kTabWaves;
        {
            const int base = 16 * b0, cnt = min(16 * b1, nc) - base;   // <= 128
            // one stable counting pass by the row pair (pk >> 5) & 3 (ballots
            // + mbcnt, in the wave's own part of the list)
            constexpr int SH = 5, NBINS = 4;
            int2 e0 = make_int2(0, 0), e1 = make_int2(0, 0);
            int bin0 = NBINS, bin1 = NBINS;
            if (lane < cnt) { e0 = cand[base + lane]; bin0 = (e0.y >> SH) & (NBINS - 1); }
            if (lane + 64 < cnt) { e1 = cand[base + 64 + lane]; bin1 = (e1.y >> SH) & (NBINS - 1); }
            int r0 = 0, r1 = 0, run = 0;
            static_for<NBINS>([&](auto Yc) {
                constexpr int y = Yc;
                const uint64_t m0 = __ballot(bin0 == y), m1 = __ballot(bin1 == y);
                const int p0 = __popcll(m0);
                if (bin0 == y) r0 = run + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
                if (bin1 == y) r1 = run + p0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
                run += p0 + __popcll(m1);
            });
            if (lane < cnt) cand[base + r0] = e0;
            if (lane + 64 < cnt) cand[base + r1] = e1;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        TSTAMP(ts2);
        // ---- 3. + 4. units of two M-blocks (32 consecutive sorted candidates) ----
        for (int fb = b0; fb < b1; fb += 2) {
            const int nh = min(2, b1 - fb);
            auto unit = [&](auto nhc) {
                constexpr int NH = decltype(nhc)::value;
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
                // row 0 of the wave: each candidate's table row, published for
                // the epilogue's lanes; its own S_a and w_a from the tables
                int sa_raw[NH];
                double wa_raw[NH];
#pragma unroll
                for (int h = 0; h < NH; ++h) { sa_raw[h] = 0; wa_raw[h] = 0.0; }
                if (kh == 0) {
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const int tix = tix0 + (rrel[h] * sc.W + qrel[h]) * VP;
                        ti[16 * h + m].tix = tix;
                        ti[16 * h + m].R = valid[h] ? Rv[h] : -1;
                        sa_raw[h] = tsb[tix + Rv[h]];
                        wa_raw[h] = tw[tix + Rv[h]];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                // the epilogue's table values, one candidate step ahead: lane
                // (kh, m) needs candidate 4 kh + i's S_b and w_b of views 16 nb + m
                double sacc[NH][4];
                int sbv[2][NH][NBLK];
                double wv[2][NH][NBLK];
                auto fetch = [&](auto ic) {
                    constexpr int i = decltype(ic)::value;
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const int tix = ti[16 * h + 4 * kh + i].tix + m;
#pragma unroll
                        for (int nb = 0; nb < NBLK; ++nb) {
                            sbv[i & 1][h][nb] = tsb[tix + 16 * nb];
                            wv[i & 1][h][nb] = tw[tix + 16 * nb];
                        }
                    }
                };
                TSTAMP(tk0);
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
                // NST K-steps from sb; steps below sd are done (their A rows read
                // zeros); steps [SAFE_LO, SAFE_HI] hold window rows of every
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
                    uint4 av[2][NH], bv[2][NBLK];
                    auto load = [&](int st, int slot) {
#pragma unroll
                        for (int h = 0; h < NH; ++h)
                            av[slot][h] = *(const uint4*)(reg + ((st >= SAFE_LO && st <= SAFE_HI) ||
                                                                         ((rbp[h] >> (2 * st)) & 1u)
                                                                     ? aoff[h] + 64 * st : zoff));
#pragma unroll
                        for (int nb = 0; nb < NBLK; ++nb) bv[slot][nb] = *(const uint4*)(bptr[nb] + 64 * st);
                    };
                    load(0, 0);
#pragma unroll
                    for (int st = 0; st < NST; ++st) {
                        const int cs = st & 1;
                        if (st + 1 < NST) load(st + 1, cs ^ 1);
                        v4i A[NH];
#pragma unroll
                        for (int h = 0; h < NH; ++h)
                            A[h] = (v4i){(int)(av[cs][h].x & cm[h][0]), (int)(av[cs][h].y & cm[h][1]),
                                         (int)(av[cs][h].z & cm[h][2]), (int)(av[cs][h].w & cm[h][3])};
#pragma unroll
                        for (int nb = 0; nb < NBLK; ++nb) {
                            const v4i B = {(int)bv[cs][nb].x, (int)bv[cs][nb].y, (int)bv[cs][nb].z, (int)bv[cs][nb].w};
#pragma unroll
                            for (int h = 0; h < NH; ++h)
                                C[h][nb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[h], B, C[h][nb], 0, 0, 0);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
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
                TSTAMP(tk1);
                TSTAMP_ADD(5, tk1 - tk0);
                // the first candidate step's table values (issued after the K-loop:
                // in flight across it they would hold 18 registers)
                fetch(std::integral_constant<int, 0>{});
                // the candidates' decision constants (row 0), now that S_a, w_a are in
                double my_wa[NH];
#pragma unroll
                for (int h = 0; h < NH; ++h) my_wa[h] = 0.0;
                if (kh == 0) {
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const double wa = wa_raw[h];
                        ti[16 * h + m].Sa = -sa_raw[h];
                        // FAST: T = thr (n-1)/n sqrt(da) (binary32: a 1-ulp
                        // reciprocal, well inside the guard band); else the
                        // decision is on ncc
                        ti[16 * h + m].T = FAST ? (valid[h] ? tqf * __builtin_amdgcn_rcpf((float)wa) : __builtin_nanf(""))
                                                : 0.0f;
                        my_wa[h] = wa;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                // lane (kh, m) holds C[h][nb][i] = block h's candidate 4 kh + i, view 16 nb + m
                uint32_t pmv[NH], gdv[NH];
#pragma unroll
                for (int h = 0; h < NH; ++h) pmv[h] = gdv[h] = 0u;
                static_for<4>([&](auto Ic) {
                    constexpr int i = Ic;
                    if constexpr (i < 3) fetch(std::integral_constant<int, i + 1>{});
#pragma unroll
                    for (int h = 0; h < NH; ++h) {
                        const TabInfo c = ti[16 * h + 4 * kh + i];
                        const float gT = 2e-6f * fabsf(c.T);
                        float ax[NBLK];
                        double ca = 0.0;
                        const int cR = c.R;
                        if constexpr (!FAST) ca = cR < 0 ? 0.0 : kn * tw[c.tix + cR];
                        double sa = 0.0;
                        uint64_t g = 0;
                        static_for<NBLK>([&](auto Nc) {
                            constexpr int nb = Nc;
                            const int vl = 16 * nb + m;
                            const int num = __mul24(c.Sa, sbv[i & 1][h][nb]) + __mul24(NPX, C[h][nb][i]);
                            uint64_t P;
                            if constexpr (FAST) {
                                const double w = wv[i & 1][h][nb];
                                // ncc > thr <=> num w_b > T; a constant window (w_b nan)
                                // never passes.  The candidate's own view R passes (its ncc
                                // is n/(n-1) > thr): its mask bit and its term of the sum
                                // are taken out once per candidate
                                const float x = fmaf((float)num, (float)w, -c.T);
                                P = __builtin_amdgcn_fcmpf(x, 0.0f, 2);                         // ogt
                                ax[nb] = x;
                                sa = fma_f64_lanes(sa, num, w, P);
                            } else {
                                const double w = wv[i & 1][h][nb];
                                const double ncc = (double)num * w * ca;
                                const bool pass = vl != cR && ncc > a.thr;
                                P = __ballot(pass);
                                g |= __ballot(vl != cR && fabs(ncc - a.thr) <= kGuard);
                                sa = fma((double)num, pass ? w : 0.0, sa);
                            }
                            pmv[h] = writelane<2 * (i * NBLK + nb)>(pmv[h], (uint32_t)P);
                            pmv[h] = writelane<2 * (i * NBLK + nb) + 1>(pmv[h], (uint32_t)(P >> 32));
                        });
                        if constexpr (FAST) {
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
                // bits, guard bits and sum from the lanes that hold them
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
                        double av = 0.0;
                        if (a.avg) {
                            // its own term num_RR w_a = D_a w_a = 1 / w_a leaves the sum
                            double inv = __builtin_amdgcn_rcp(my_wa[h]);
                            inv = inv * (2.0 - my_wa[h] * inv);
                            const double sum = self ? mine - inv : mine;
                            av = cnt ? sum * (kn * my_wa[h]) * s_recip[cnt] : 0.0;
                        }
                        if (a.rec) {
                            // one 16-B record [mask word, avg] (|V| = popcount)
                            const unsigned long long ab = __double_as_longlong(av);
                            *(uint4*)(a.mask + 2 * idx) = make_uint4((uint32_t)mk, (uint32_t)(mk >> 32), (uint32_t)ab,
                                                                     (uint32_t)(ab >> 32));
                        } else {
                            a.mask[idx] = mk;
                            a.count[idx] = cnt;
                            if (a.avg) a.avg[idx] = av;
                        }
                        if (gg) t.fix_list[atomicAdd(t.fix_count, 1)] = make_int4((int32_t)idx, dcur.x, e[h].y, 0);
                    }
                }
                TSTAMP(tk2);
                TSTAMP_ADD(6, tk2 - tk1);
            };
            if (nh == 2) unit(std::integral_constant<int, 2>{});
            else unit(std::integral_constant<int, 1>{});
            TSTAMP_ADD(4, nh);
            // thread 0 claims item k+2 after wave 0's first unit: less held
            // back when the queue runs dry
            if (fb == b0 && tid == 0 && nx1 < n_units) pend = claim();
        }
        if (b0 >= b1 && tid == 0 && nx1 < n_units) pend = claim();
        TSTAMP(ts3);
        if (wave == 0) TSTAMP_ADD(0, 1);
        TSTAMP_ADD(1, ts1 - ts0);
        TSTAMP_ADD(2, ts2 - ts1);
        TSTAMP_ADD(3, ts3 - ts2);
        if (nx1 >= n_units) return false;
        if constexpr (!DB) {
            // one buffer: every wave is done with it before the next item lands
            __syncthreads();
            stage(dst1, std::integral_constant<int, 0>{});
        }
        cur = nx1;
        dcur = desc(it1, c1);
        return true;
    };
    for (;;) {
        if (!round(std::integral_constant<int, 0>{})) break;
        if (!round(std::integral_constant<int, DB ? 1 : 0>{})) break;
    }
#ifdef MVS_STAMPS
    // the workgroup's start and end on the 100 MHz clock (slots 10, 11; thread 0)
    if (tid == 0) {
        atomicAdd(&g_stamps_tab[(blockIdx.x & 1023) * 16 + 10], (unsigned long long)t_wg0);
        atomicAdd(&g_stamps_tab[(blockIdx.x & 1023) * 16 + 11], (unsigned long long)__builtin_amdgcn_s_memrealtime());
        // where it ran: HW_ID (CU, SH, SE) and XCC_ID, + 1 (slots 12, 13)
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
        atomicAdd(&g_stamps_tab[(blockIdx.x & 1023) * 16 + 12], (unsigned long long)hw + 1ull);
        atomicAdd(&g_stamps_tab[(blockIdx.x & 1023) * 16 + 13], (unsigned long long)xcc + 1ull);
    }
#endif
}


// hipFuncAttributeMaxDynamicSharedMemorySize is not needed: all LDS is static
template <int WID, int NBLK>
int launch_tab(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, const MomentsDev* mt, hipStream_t s) {
    const dim3 grid(t->grid > 0 ? std::min(t->grid, kTabGrid) : kTabGrid);
    if (fabs(a->thr) >= 0.01)
        hipLaunchKernelGGL((k_score_tab<WID, NBLK, true>), grid, dim3(kTabThreads), 0, s, *sc, *a, *t, *mt,
                           (const int4*)t->items, (const int2*)t->sorted);
    else
        hipLaunchKernelGGL((k_score_tab<WID, NBLK, false>), grid, dim3(kTabThreads), 0, s, *sc, *a, *t, *mt,
                           (const int4*)t->items, (const int2*)t->sorted);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int WID>
int launch_tab_w(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, const MomentsDev* mt, hipStream_t s) {
    switch ((sc->V + 15) / 16) {
        case 1: return launch_tab<WID, 1>(sc, a, t, mt, s);
        case 2: return launch_tab<WID, 2>(sc, a, t, mt, s);
        case 3: return launch_tab<WID, 3>(sc, a, t, mt, s);
        default: return launch_tab<WID, 4>(sc, a, t, mt, s);
    }
}

}  // namespace

#ifdef MVS_STAMPS
extern "C" int mvs_read_stamps_tab(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_tab), sizeof(g_stamps_tab)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int mvs_launch_moments(const SceneDev* sc, const MomentsDev* mt, hipStream_t s) {
    const bool dtab = moments_dtab(sc->V);
    if (mt->VP != (sc->V > 64 ? 64 * ((sc->V + 63) / 64) : 16 * ((sc->V + 15) / 16))) return -3;
    const dim3 grid((unsigned)((sc->W + kMomW - 1) / kMomW), (unsigned)((sc->H + kMomH - 1) / kMomH),
                    (unsigned)(mt->VP / kMomV));
#define MVS_MOM(W_) (dtab ? (const void*)k_moments<W_, true> : (const void*)k_moments<W_, false>)
    const void* f = nullptr;
    switch (mt->wid) {
        case 1: f = MVS_MOM(1); break;
        case 2: f = MVS_MOM(2); break;
        case 3: f = MVS_MOM(3); break;
        case 4: f = MVS_MOM(4); break;
        case 5: f = MVS_MOM(5); break;
        default: return -2;
    }
#undef MVS_MOM
    const SceneDev scv = *sc;
    const MomentsDev mtv = *mt;
    void* args[] = {(void*)&scv, (void*)&mtv};
    if (hipLaunchKernel(f, grid, dim3(256), args, 0, s) != hipSuccess) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mvs_launch_score_tab(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, const MomentsDev* mt,
                                    hipStream_t s) {
    if (sc->V > 64 || t->chunk != kTabChunk) return -3;
    switch (mt->wid) {
        case 1: return launch_tab_w<1>(sc, a, t, mt, s);
        case 2: return launch_tab_w<2>(sc, a, t, mt, s);
        case 3: return launch_tab_w<3>(sc, a, t, mt, s);
        case 4: return launch_tab_w<4>(sc, a, t, mt, s);
        case 5: return launch_tab_w<5>(sc, a, t, mt, s);
        default: return -2;
    }
}

// Device helpers of the tiled matrix-core scorers (k_score_mma, k_score_mma_v
// in mvs_kernels.hip; k_score_tab in mvs_score_tab.hip): the tile geometry,
// the i8 MFMA operand masks, EXEC-masked binary64 accumulation, lane moves
// and reductions.  gfx950 only.
#pragma once
#include <utility>

#include "mvs_device.h"

namespace {

// Binary64 DPP move (both halves), bound_ctrl: every source lane exists.
template <int CTRL>
DEV double dpp_f64(double x) {
    const unsigned long long u = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Reduce-scatter of four values over each row of 16 lanes: lane m of a row
// (m = lane & 15) returns the row sum of x[m & 3], so lanes m < 4 hold the
// four sums.  Two partner swaps halve the values a lane carries (keep one
// index, send the other), then two rotations sum the lanes that share the low
// two bits: 27 VALU instead of four full row sums (48) and a select.
DEV double row_sum16_x4(const double (&x)[4], int m) {
    const bool b0 = m & 1, b1 = (m >> 1) & 1;
    double k0 = b0 ? x[1] : x[0], s0 = b0 ? x[0] : x[1];
    double k1 = b0 ? x[3] : x[2], s1 = b0 ? x[2] : x[3];
    k0 += dpp_f64<0xB1>(s0);    // quad_perm [1,0,3,2]: index b0 (+2)
    k1 += dpp_f64<0xB1>(s1);
    double kk = b1 ? k1 : k0;
    const double ss = b1 ? k0 : k1;
    kk += dpp_f64<0x4E>(ss);    // quad_perm [2,3,0,1]: index b0 + 2 b1
    kk += dpp_f64<0x124>(kk);   // row_ror:4
    kk += dpp_f64<0x128>(kk);   // row_ror:8
    return kk;
}

typedef int v4i __attribute__((ext_vector_type(4)));

template <int WID>
struct MmaGeom {
    static constexpr int NB = 2 * WID + 1;
    static constexpr int NPX = NB * NB;
    static constexpr int ROWS = MVS_TILE_H + 2 * WID;   // region rows (even)
    static constexpr int KS = ROWS / 2;                 // K-steps of two region rows
    static constexpr int VS = ROWS * 32 + 32;           // bytes per view: VS/16 = 2 mod 4, so the
                                                        // B reads (ds_read_b128) are conflict-free
    static constexpr int C0 = 8 - WID;                  // region column of the first window column of x0
    static_assert(C0 >= 0 && C0 + MVS_TILE_W - 1 + NB <= 32, "window must fit the 32 region columns");
    static_assert(ROWS % 2 == 0, "K-steps take two rows");
};

// x through an opaque copy: what is computed from it is computed where it is
// used, not hoisted out of loops into long-lived registers
DEV int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Band queues of a persistent scorer: work items [0, n) in nb contiguous
// bands, band x's head at heads[32 x]; the first skip(x) items of band x are
// handed out without a claim.  A workgroup claims from band cb (its own band
// first) and moves to the next band when that one is exhausted; n: none left.
template <class Skip>
DEV int band_claim(int32_t* heads, int& cb, int ob, int nb, int n, Skip&& skip) {
    for (; cb < ob + nb; ++cb) {
        const int x = cb % nb;
        const int lo = (int)((int64_t)n * x / nb), hi = (int)((int64_t)n * (x + 1) / nb);
        const int r = atomicAdd(heads + 32 * x, 1) + skip(x);
        if (r < hi - lo) return lo + r;
    }
    return n;
}

// acc += num * w in the lanes of P only (binary64): EXEC narrowed to P for
// the conversion and the fma, restored after -- two vector instructions, no
// select of the term (the compiler's form of the select costs four)
// the same on a binary64 num (converted once, shared with the decision)
DEV double fma_f64_lanes_d(double acc, double num, double w, uint64_t P) {
    uint64_t save;
    asm volatile(
        "s_and_saveexec_b64 %[save], %[p]\n\t"
        "v_fma_f64 %[acc], %[num], %[w], %[acc]\n\t"
        "s_mov_b64 exec, %[save]"
        : [acc] "+v"(acc), [save] "=&s"(save)
        : [num] "v"(num), [w] "v"(w), [p] "s"(P)
        : "scc");   // EXEC is restored before the statement ends
    return acc;
}
DEV double fma_f64_lanes(double acc, int num, double w, uint64_t P) {
    double t;
    uint64_t save;
    asm volatile(
        "s_and_saveexec_b64 %[save], %[p]\n\t"
        "v_cvt_f64_i32 %[t], %[num]\n\t"
        "v_fma_f64 %[acc], %[t], %[w], %[acc]\n\t"
        "s_mov_b64 exec, %[save]"
        : [acc] "+v"(acc), [t] "=&v"(t), [save] "=&s"(save)
        : [num] "v"(num), [w] "v"(w), [p] "s"(P)
        : "scc");   // EXEC is restored before the statement ends
    return acc;
}

// 4-bit column mask -> byte mask
DEV uint32_t byte_mask(uint32_t nib) { return ((nib * 0x00204081u) & 0x01010101u) * 0xffu; }

// 1/k for k = 0..64 (entry 0 unused), correctly rounded at compile time
struct RecipTable {
    double r[65];
    constexpr RecipTable() : r() {
        for (int k = 1; k <= 64; ++k) r[k] = 1.0 / (double)k;
    }
};
__constant__ constexpr RecipTable c_recip{};

// v_writelane_b32 (lane LANE of v takes the wave-uniform x) through the LLVM
// intrinsic, so that the hazard recognizer sees it: a VALU write of the
// source SGPR (a ballot's v_cmp) needs wait states before v_writelane reads
// it, which inline asm would hide from the compiler
extern "C" __device__ int mvs_llvm_writelane(int x, int lane, int v) __asm("llvm.amdgcn.writelane.i32");
template <int LANE>
DEV uint32_t writelane(uint32_t v, uint32_t x) {
    return (uint32_t)mvs_llvm_writelane((int)x, LANE, (int)v);
}

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N-1>)
template <class F, int... I>
DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
DEV void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Work item v of the tiled scorers: (tile, first bucket entry, candidates)
// from the item list's (tile, chunk j) and the tile's final count
// (uniform: scalar loads)
// The work items in kItemSegs segments (k_item_scan fills segment 0; the
// layout also takes per-workgroup appends, one n_items atomic per
// workgroup and segment, not one chain over the whole grid), as one list:
// item v of the list is entry v - pre[x] of segment x, pre[x] <= v < pre[x+1]
struct ItemMap {
    int pre[kItemSegs + 1];
    int seg;
    DEV void load(const TiledArgs& t) {
        pre[0] = 0;
#pragma unroll
        for (int x = 0; x < kItemSegs; ++x) pre[x + 1] = pre[x] + t.n_items[32 * x];
        seg = t.item_seg;
    }
    DEV int total() const { return pre[kItemSegs]; }
    DEV int slot(int v) const {
        int s = v;
#pragma unroll
        for (int x = 1; x < kItemSegs; ++x)
            if (v >= pre[x]) s = x * seg + v - pre[x];
        return s;
    }
};

DEV int4 item_desc(const TiledArgs& t, const int4* __restrict__ items, const ItemMap& im, int v) {
    const int4 it = items[im.slot(v)];
    const int cnt = min(t.tile_count[it.x * kTcStride], t.cap);
    return make_int4(it.x, it.x * t.cap + it.y * t.chunk, min(cnt - it.y * t.chunk, t.chunk), 0);
}

// Workgroup barrier for LDS traffic: every wave's LDS operations are complete
// first; outstanding global loads and LDS-DMA are not waited for (the fence of
// __syncthreads would wait for them: vmcnt(0)).
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


}  // namespace

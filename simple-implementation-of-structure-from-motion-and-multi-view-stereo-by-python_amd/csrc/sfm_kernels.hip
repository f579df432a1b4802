// SfM front-end kernels (gfx950): Harris keypoints and NCC descriptor
// matching -- the producer of the MVS stage's seed tracks (HarrisFeatures.py,
// SFM.py).  Reads the scene's view-major gray copy
// (SceneDev::gv).
#include <algorithm>
#include <cmath>

#include "mvs_device.h"

namespace {

DEV int refl101(int i, int n) {     // BORDER_REFLECT_101 for overruns of <= n - 1
    return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

DEV float gv_px(const SceneDev& sc, int v, int y, int x) {
    return (float)(sc.gv[((int64_t)v * sc.H + y) * sc.Wp + x] ^ 0x80u);   // gv holds g - 128
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
                    const uint32_t g = sc.gv[((int64_t)v * sc.H + r - wid + p / nb) * sc.Wp + q - wid + p % nb] ^ 0x80u;
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

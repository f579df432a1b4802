// Host side of libmvs_amd.so: scene context, camera table, seeding, the
// ordered expansion commit engine and the C-ABI of include/mvs_amd.h.
//
// Reference: MVS2.py:176-404 (DensePointsWithMVS2, patch_expansion,
// CellTable), utils.py:234-254 (geometry helpers).
//
// Design.  Everything a candidate's photo test and accept test depend on is
// immutable (parent patch, cameras, images), so scoring runs speculatively on
// the GPU in sweeps; only the cell-table vacancy checks, the FIFO order, the
// `break` of the j loop and the pop cap are order dependent, and those are
// replayed here on the host exactly in reference order.  A patch's children
// -- (hit view, i in {-1,+1}); the geometry does not depend on j
// (MVS2.py:334) -- are scored once per distinct record and memoised.
//
// Compiled with -ffp-contract=off: host geometry (Jacobi SVD, triangulation,
// camera constants) follows OpenCV's / numpy's operation order.
#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mvs_amd.h"
#include "mvs_internal.h"

namespace {

thread_local std::string g_err;

struct Fail {
    int code;
    std::string msg;
};

#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess)                                                             \
            throw Fail{MVS_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)};        \
    } while (0)

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        release();
        if (count == 0) count = 1;
        HIPCHK(hipMalloc((void**)&p, count * sizeof(T)));
        n = count;
    }
    void ensure(size_t count) {
        if (count > n) alloc(std::max(count, n * 2));
    }
    // grow preserving the first `keep` elements
    void grow(size_t count, size_t keep, hipStream_t s) {
        if (count <= n) return;
        T* q = nullptr;
        size_t nn = std::max(count, n * 2);
        HIPCHK(hipMalloc((void**)&q, nn * sizeof(T)));
        if (p && keep) HIPCHK(hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        release();
        p = q;
        n = nn;
    }
};

// ---------------------------------------------------------------------------
// Host geometry (OpenCV 4.x algorithms the reference calls through cv2)
// ---------------------------------------------------------------------------

// cv::JacobiSVDImpl_<double>: one-sided Jacobi on the n rows (length m) of At.
void jacobi_svd(double* At, double* Wout, double* Vt, int m, int n) {
    double W[16];
    const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
    const int max_iter = std::max(m, 30);
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const double t = At[i * m + k];
            sd += t * t;
        }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double* Ai = At + i * m;
                double* Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = std::hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = std::sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = std::sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                double* Vi = Vt + i * n;
                double* Vj = Vt + j * n;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vi[k] + s * Vj[k];
                    const double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const double t = At[i * m + k];
            sd += t * t;
        }
        W[i] = std::sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            std::swap(W[i], W[j]);
            for (int k = 0; k < m; k++) std::swap(At[i * m + k], At[j * m + k]);
            for (int k = 0; k < n; k++) std::swap(Vt[i * n + k], Vt[j * n + k]);
        }
    }
    for (int i = 0; i < n; i++) Wout[i] = W[i];
    for (int i = 0; i < n; i++) {
        const double s = W[i] > minval ? 1 / W[i] : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

// cvRodrigues2 3x3 -> 3x1 then 3x1 -> 3x3 (projectPoint, utils.py:242-243).
void rodrigues_roundtrip(const double* Rin, double* Rout) {
    double At[9], W[3], Vt[9], U[9], R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) At[i * 3 + j] = Rin[j * 3 + i];
    jacobi_svd(At, W, Vt, 3, 3);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) U[i * 3 + j] = At[j * 3 + i];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += U[i * 3 + k] * Vt[k * 3 + j];
            R[i * 3 + j] = s;
        }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = std::sqrt(std::max(t, 0.));
            t = (R[4] + 1) * 0.5;
            ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) &&
                (R[5] > 0) != (ry * rz > 0))
                rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta;
            ry *= theta;
            rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    // 3x1 -> 3x3
    const double th = std::sqrt(rx * rx + ry * ry + rz * rz);
    if (th < DBL_EPSILON) {
        for (int i = 0; i < 9; i++) Rout[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    // glibc sincos(): the gcc -O2 lowering of OpenCV's adjacent cos/sin calls
    double ss, cc;
    ::sincos(th, &ss, &cc);
    const double c1 = 1. - cc;
    const double ith = th ? 1. / th : 0.;
    rx *= ith;
    ry *= ith;
    rz *= ith;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int i = 0; i < 9; i++) {
        const double e = (i % 4 == 0) ? 1.0 : 0.0;
        Rout[i] = (cc * e + c1 * rrt[i]) + ss * r_x[i];
    }
}

// cvTriangulatePoints for one correspondence (utils.py:238-239).
void triangulate(const double* P1, const double* P2, const double* x1, const double* x2, double* X4) {
    double A[16];
    const double* P[2] = {P1, P2};
    const double* pt[2] = {x1, x2};
    for (int j = 0; j < 2; j++) {
        const double x = pt[j][0], y = pt[j][1];
        for (int k = 0; k < 4; k++) {
            A[(j * 2 + 0) * 4 + k] = x * P[j][8 + k] - P[j][0 + k];
            A[(j * 2 + 1) * 4 + k] = y * P[j][8 + k] - P[j][4 + k];
        }
    }
    double At[16], W[4], Vt[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) At[i * 4 + j] = A[j * 4 + i];
    jacobi_svd(At, W, Vt, 4, 4);
    for (int k = 0; k < 4; k++) X4[k] = Vt[12 + k];
}

inline double fma_dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
    // numpy 3-element dot / matvec row as OpenBLAS 0.3.29 evaluates it
    return std::fma(a2, b2, std::fma(a1, b1, a0 * b0));
}

inline int py_wrap(long i, long n) { return (int)(i < 0 ? i + n : i); }

// cv2.projectPoints of one point, no distortion (cvProjectPoints2Internal
// order; the device project() in mvs_kernels.hip is the same expression)
void project_host(const double* K, const double* Rp, const double* t, const double* M, double* out) {
    double x = Rp[0] * M[0] + Rp[1] * M[1] + Rp[2] * M[2] + t[0];
    double y = Rp[3] * M[0] + Rp[4] * M[1] + Rp[5] * M[2] + t[1];
    double z = Rp[6] * M[0] + Rp[7] * M[1] + Rp[8] * M[2] + t[2];
    z = z != 0.0 ? 1.0 / z : 1.0;
    x *= z;
    y *= z;
    out[0] = x * K[0] + K[2];
    out[1] = y * K[4] + K[5];
}

// getProjectionMatrix(K, R, t) = K @ [R | t] (utils.py:234-236) as OpenBLAS
// evaluates the 3x3 by 3x4 product: an FMA chain per entry
void projection_matrix(const double* K, const double* R, const double* t, double* P) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) {
            const double e0 = c < 3 ? R[c] : t[0], e1 = c < 3 ? R[3 + c] : t[1],
                         e2 = c < 3 ? R[6 + c] : t[2];
            P[4 * r + c] = fma_dot3(K[3 * r], K[3 * r + 1], K[3 * r + 2], e0, e1, e2);
        }
}

}  // namespace

// ---------------------------------------------------------------------------
// Context
// ---------------------------------------------------------------------------

struct mvs_ctx {
    int device = 0;
    int stage_flags = 0;   // mvs_stage_set_options
    int V = 0, H = 0, W = 0, Wq = 0;
    hipStream_t stream = nullptr;
    std::vector<CamDev> cams;
    std::vector<double> K;   // V*9 as given (getProjectionMatrix uses all of K)
    std::vector<uint8_t> h_rgb;
    DevBuf<uint8_t> d_rgb, d_stack, d_gv;
    DevBuf<CamDev> d_cams;
    DevBuf<int32_t> d_exact;
    DevBuf<unsigned long long> d_stats;   // mvs_scorer_stats (k_score_fix)
    SceneDev sc{};
    // scratch for host-pointer scoring
    DevBuf<double> s_c, s_xy, s_avg;
    DevBuf<int32_t> s_ref, s_count;
    DevBuf<uint64_t> s_mask;
    // tiled scorer scratch
    DevBuf<int32_t> t_tiles, t_cand;
    // mvs_pack_accepted: the pack's row counter and chunk ticket (k_acc_pack
    // leaves both zero)
    DevBuf<unsigned long long> p_ctl;
    DevBuf<int4> t_items;
    // SfM front-end scratch (Harris maps, descriptors, match rows)
    DevBuf<float> f_resp, f_dil;
    DevBuf<uint32_t> f_key, f_desc;
    DevBuf<int32_t> f_rows, f_pts, f_mom, f_best;
    int kernel_mode = 0;   // 0 auto, 1 direct, 2 tiled (env MVS_SCORE_KERNEL)
    // the tiled scorer's window moments: per wid, built on first use
    // (k_moments), rebuilt with the scene; tab_mode 0 = tables when they fit
    // (ring256 with tile-order items: 1.52 ms per 2^20 against 1.67-1.69 ms
    // for the in-kernel Q table), 1 = never (in-kernel moments; env
    // MVS_SCORE_KERNEL=mma), 2 = tables (env MVS_SCORE_KERNEL=tab)
    int tab_mode = 0;
    int scorer_wgs = 0;   // env MVS_SCORER_WGS: k_score_tab's grid (0 = every CU, twice)
    DevBuf<int16_t> mom_sb[MVS_MAX_WID + 1];
    DevBuf<double> mom_w[MVS_MAX_WID + 1];     // V <= 64
    DevBuf<int32_t> mom_d[MVS_MAX_WID + 1];    // V > 64 (moments_dtab)
    DevBuf<uint16_t> mom_flat[MVS_MAX_WID + 1];   // constant-window bits (MomentsDev.flat)
    bool mom_ok[MVS_MAX_WID + 1] = {};
    int moments_vp() const { return V > MVS_GROUP_VIEWS ? 64 * ((V + 63) / 64) : 16 * ((V + 15) / 16); }
    MomentsDev moments(int wid) const {
        MomentsDev m{};
        m.sb = mom_sb[wid].p;
        m.w = mom_w[wid].p;
        m.d = mom_d[wid].p;
        m.flat = mom_flat[wid].p;
        m.VP = moments_vp();
        m.wid = wid;
        return m;
    }
    // the tables of wid (10 B per (pixel, view) at V <= 64: S_b and w; 6 B at
    // V > 64: S_b and D), built on stream s if needed; false when they do not
    // apply (disabled, or more than 2^31 elements).  One row of 16 pixels
    // past the end: k_score_tab stages a tile's rows whole (16 pixels x VP),
    // also where the last tile column runs past W
    // Memory: (H W + 16) VP elements per wid, 10 B each at V <= 64 (S_b int16
    // + w binary64) or 6 B at V > 64
    // (S_b + D int32): 147 MB per wid at dinoRing, 3.2 GB at 256 x 1920 x 1080.  A scene past tab_limit elements (2^31;
    // env MVS_TAB_LIMIT lowers it, for tests) or whose tables cannot be
    // allocated is scored with the in-kernel moments instead (same results).
    int64_t tab_limit = (int64_t)1 << 31;
    bool ensure_moments(int wid, hipStream_t s) {
        if (tab_mode == 1) return false;
        const int64_t elems = ((int64_t)H * W + 16) * moments_vp();
        if (elems >= tab_limit) return false;
        if (!mom_ok[wid]) {
            try {
                mom_sb[wid].alloc((size_t)elems);
                if (moments_dtab(V)) mom_d[wid].alloc((size_t)elems);
                else mom_w[wid].alloc((size_t)elems);
                mom_flat[wid].alloc((size_t)(elems / 16));
            } catch (const Fail&) {
                mom_sb[wid].release();
                mom_d[wid].release();
                mom_w[wid].release();
                mom_flat[wid].release();
                (void)hipGetLastError();   // the failed hipMalloc's error is not this call's
                return false;
            }
            HIPCHK(hipMemsetAsync(mom_sb[wid].p, 0, (size_t)elems * sizeof(int16_t), s));
            HIPCHK(hipMemsetAsync(mom_flat[wid].p, 0, (size_t)(elems / 16) * sizeof(uint16_t), s));
            if (moments_dtab(V))
                HIPCHK(hipMemsetAsync(mom_d[wid].p, 0, (size_t)elems * sizeof(int32_t), s));
            else
                HIPCHK(hipMemsetAsync(mom_w[wid].p, 0, (size_t)elems * sizeof(double), s));
            const MomentsDev m = moments(wid);
            if (mvs_launch_moments(&sc, &m, s) != 0) throw Fail{MVS_E_HIP, "moments launch failed"};
            mom_ok[wid] = true;
        }
        return true;
    }
    int tiles_clean_ntiles = -1;   // the next batch's counter set known zero for this tile count (-1: unknown)
    int tiles_parity = 0;          // the counter set the next tiled batch uses
    // kernel timing (mvs_kernel_timing): one event pair per `timing_period`-th
    // scoring launch (an event record between two kernels costs a few us of
    // stream time, so a timed loop samples)
    bool timing = false;
    int timing_period = 1;
    int64_t timing_count = 0;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    const char* timed_name = "";   // the kernel the last timed pair bracketed
    // The context's scratch (tiled-scorer counters and lists, host-pointer
    // buffers) and the exchange pack's status words may be used on any stream
    // a *_device call names: a call waits for the previous use when the
    // stream changes.  The event is recorded then, lazily, on the stream that
    // used the area last (its later work is waited for too): consecutive
    // calls on one stream enqueue nothing, where an event record after every
    // call cost the stream ~5 us of idle time before the next call's first
    // kernel (profiles/r05/r5d_kernel_trace.csv).  A stream destroyed since
    // its use cannot take the record: the whole device is synchronised then.
    struct StreamOrder {
        hipEvent_t ev = nullptr;
        hipStream_t s = nullptr;
        bool used = false;
        void acquire(hipStream_t cur) {
            if (!used || s == cur) return;
            if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            if (hipEventRecord(ev, s) != hipSuccess) {
                (void)hipGetLastError();
                HIPCHK(hipDeviceSynchronize());
                return;
            }
            HIPCHK(hipStreamWaitEvent(cur, ev, 0));
        }
        void release(hipStream_t cur) {
            s = cur;
            used = true;
        }
        // the stream st is about to be destroyed: its work on the area is
        // waited for now, so no later acquire records an event on it
        void retire(hipStream_t st) {
            if (!used || s != st) return;
            HIPCHK(hipStreamSynchronize(st));
            used = false;
            s = nullptr;
        }
    } scratch_order, pack_order;
    std::string err;
    void scratch_acquire(hipStream_t s) { scratch_order.acquire(s); }
    void scratch_release(hipStream_t s) { scratch_order.release(s); }
    // next event pair while timing is on, else nulls
    void next_events(hipEvent_t* e0, hipEvent_t* e1) {
        *e0 = *e1 = nullptr;
        if (!timing) return;
        if (timing_count++ % timing_period) return;
        if (ev_used + 2 > ev.size()) {
            for (int k = 0; k < 2; ++k) {
                hipEvent_t e;
                // no system-scope fence at the record: no L2 writeback between
                // the timed kernels (the timestamps need none)
                HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
                ev.push_back(e);
            }
        }
        *e0 = ev[ev_used];
        *e1 = ev[ev_used + 1];
        ev_used += 2;
    }
    int words() const { return (V + 63) / 64; }
};

struct mvs_stage;
// The stage's outputs: the [x y z r g b] rows of initial_patches and
// all_patches, ordered and gathered on the device (HBM); mvs_stage_rows copies
// them straight into the caller's buffer.
struct mvs_stage_result {
    int device = 0;
    DevBuf<double> d_init, d_all;   // rows * 6
    int64_t n_init = 0, n_all = 0;
    int64_t stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double times[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // mvs_stage_times
    int64_t filt[2] = {0, 0};                      // mvs_stage_filter_stats
};

namespace {

void build_cameras(mvs_ctx* ctx, const double* K, const double* R, const double* t, const double* Rp) {
    ctx->cams.resize(ctx->V);
    for (int v = 0; v < ctx->V; ++v) {
        CamDev& c = ctx->cams[v];
        std::memset(&c, 0, sizeof c);
        const double* Kv = K + 9 * v;
        const double* Rv = R + 9 * v;
        const double* tv = t + 3 * v;
        if (Rp)
            std::memcpy(c.Rp, Rp + 9 * v, sizeof c.Rp);
        else
            rodrigues_roundtrip(Rv, c.Rp);
        std::memcpy(c.t, tv, sizeof c.t);
        std::memcpy(c.R, Rv, sizeof c.R);
        c.fx = Kv[0];
        c.fy = Kv[4];
        c.cx = Kv[2];
        c.cy = Kv[5];
        c.fbar = (Kv[0] + Kv[4]) / 2;
        for (int j = 0; j < 3; ++j) {
            // camera_pos = -(R^T @ t) (MVS2.py:189); C = (-R^T) @ t (MVS2.py:351)
            c.O[j] = -fma_dot3(Rv[j], Rv[3 + j], Rv[6 + j], tv[0], tv[1], tv[2]);
            c.C[j] = fma_dot3(-Rv[j], -Rv[3 + j], -Rv[6 + j], tv[0], tv[1], tv[2]);
        }
    }
}

int set_err(mvs_ctx* ctx, const Fail& f) {
    if (ctx) ctx->err = f.msg;
    g_err = f.msg;
    return f.code;
}

template <class Fn>
int guarded(mvs_ctx* ctx, Fn&& fn) {
    try {
        if (ctx) HIPCHK(hipSetDevice(ctx->device));
        return fn();
    } catch (const Fail& f) {
        return set_err(ctx, f);
    } catch (const std::bad_alloc&) {
        return set_err(ctx, Fail{MVS_E_NOMEM, "host allocation failed"});
    } catch (const std::exception& e) {
        return set_err(ctx, Fail{MVS_E_ARG, e.what()});
    }
}

// d_count == null: d_mask holds records [mask words, avg bits] of words + 1
// int64 each (mvs_score_device_rec), d_avg is ignored
void score_device(mvs_ctx* ctx, int64_t n, const double* d_c, const int32_t* d_ref, int wid,
                  double thr, double* d_xy, uint64_t* d_mask, int32_t* d_count, double* d_avg,
                  hipStream_t s) {
    if (wid < 1 || wid > MVS_MAX_WID) throw Fail{MVS_E_UNSUPPORTED, "wid must be in 1..5"};
    ScoreArgs a{};
    a.n = n;
    a.c = d_c;
    a.ref = d_ref;
    a.thr = thr;
    a.xy = d_xy;
    a.mask = d_mask;
    a.count = d_count;
    a.avg = d_avg;
    a.exact_hits = ctx->d_exact.p;
    a.mstride = ctx->words();
    a.astride = 1;
    a.rec = 0;
    if (!d_count) {
        a.rec = 1;
        a.mstride = a.astride = ctx->words() + 1;
        a.avg = (double*)(d_mask + ctx->words());
    }
    // the tiled matrix-core scorer (k_score_mma, any V <= 256) for batches of
    // >= 2048 candidates; the direct k_score for small batches
    const bool grouped = ctx->V > MVS_GROUP_VIEWS;
    const bool tiled = ctx->kernel_mode == 2 || (ctx->kernel_mode == 0 && n >= 2048);
    if (tiled) {
        TiledArgs t{};
        t.tw = MVS_TILE_W;
        t.th = MVS_TILE_H;
        t.ntx = (ctx->W + MVS_TILE_W - 1) / MVS_TILE_W;
        t.nty = (ctx->H + MVS_TILE_H - 1) / MVS_TILE_H;
        const int ntiles = t.ntx * t.nty;
        const int32_t* tiles_before = ctx->t_tiles.p;
        const int64_t set_words = tc_words(ntiles);
        ctx->t_tiles.ensure((size_t)(2 * set_words));   // two counter sets (parities)
        if (ctx->t_tiles.p != tiles_before) ctx->tiles_clean_ntiles = -1;
        const int groups = grouped ? (ctx->V + MVS_GROUP_VIEWS - 1) / MVS_GROUP_VIEWS : 1;
        // tile buckets of cap candidates (16x the mean load, at least 1024:
        // expansion sweeps crowd onto the object's tiles; the rest of a tile
        // goes to the direct path), and the direct path's list (int4 entries).
        // Only the filled part of a bucket is ever touched.
        const int64_t mean = (n + ntiles - 1) / ntiles;
        int64_t cap = std::min<int64_t>(std::max<int64_t>(16 * mean, 1024), std::max<int64_t>(n, 64));
        cap = (cap + 63) & ~(int64_t)63;
        if ((int64_t)ntiles * cap >= ((int64_t)1 << 31)) cap = (((int64_t)1 << 31) - 1) / ntiles & ~(int64_t)63;
        if (cap < 64) throw Fail{MVS_E_UNSUPPORTED, "image too large for the tile buckets"};
        ctx->t_cand.ensure((size_t)2 * ntiles * cap + 4 * (size_t)n);
        t.ntiles = ntiles;
        t.cap = (int)cap;
        t.chunk = grouped ? MVS_GROUP_CHUNK : MVS_MMA_CHUNK;
        t.groups = groups;
        // this batch's counter set; k_bin zeroes the other (the previous
        // batch's) for the next batch
        int32_t* set = ctx->t_tiles.p + ctx->tiles_parity * set_words;
        t.tile_count = set;
        int32_t* ctl = set + (int64_t)ntiles * kTcStride;   // one 128-B line per counter
        t.head = ctl;
        t.fix_count = ctl + 32;
        t.n_items = ctl + 96;
        t.zero_blk = ctx->t_tiles.p + (1 - ctx->tiles_parity) * set_words;
        t.zero_words = set_words;
        t.sorted = (int2*)ctx->t_cand.p;
        t.fix_list = (int4*)(ctx->t_cand.p + 2 * (size_t)ntiles * cap);
        // at most one partial chunk per tile beyond the full ones, in any one
        // of the kItemSegs segments
        t.item_seg = (int)(n / std::max(t.chunk, 1) + ntiles + 2);
        ctx->t_items.ensure((size_t)kItemSegs * t.item_seg);
        t.items = ctx->t_items.p;
        t.zero_first = ctx->tiles_clean_ntiles != ntiles ? 1 : 0;
        t.grid = ctx->scorer_wgs;
        t.stats = ctx->d_stats.p;
        ctx->tiles_clean_ntiles = -1;            // dirty until the sequence is queued
        hipEvent_t e0, e1;
        ctx->next_events(&e0, &e1);
        ctx->scratch_acquire(s);
        const bool tab = ctx->ensure_moments(wid, s);
        const MomentsDev mt = ctx->moments(wid);
        const int rc = mvs_launch_score_tiled(&ctx->sc, &a, &t, wid, tab ? &mt : nullptr, s, e0, e1);
        if (rc != 0) throw Fail{rc == -3 ? MVS_E_UNSUPPORTED : MVS_E_HIP, "tiled score launch failed"};
        ctx->scratch_release(s);
        if (e0) ctx->timed_name = mvs_timed_kernel_name(ctx->V, wid, tab && !grouped ? 2 : 1);
        ctx->tiles_clean_ntiles = ntiles;        // the next batch's set was zeroed by this k_bin
        ctx->tiles_parity ^= 1;
        return;
    }
    hipEvent_t e0, e1;
    ctx->next_events(&e0, &e1);
    if (mvs_launch_score(&ctx->sc, &a, wid, s, e0, e1) != 0) throw Fail{MVS_E_HIP, "score launch failed"};
    if (e0) ctx->timed_name = mvs_timed_kernel_name(ctx->V, wid, 0);
}

// patch_expansion children (MVS2.py:329-369) of a.n jobs into records
// a.first_out + [0, a.n): small batches one wave per child (k_expand), large
// ones as child geometry, the children's photo test on the tiled matrix-core
// scorer, then the accept test
void expand_device(mvs_ctx* ctx, const RecordsDev& r, const ExpandArgs& a, int wid, hipStream_t s) {
    if (a.n <= 0) return;
    if (ctx->kernel_mode == 1 || a.n < 2048) {
        if (mvs_launch_expand(&ctx->sc, r, &a, wid, s) != 0) throw Fail{MVS_E_HIP, "expand launch failed"};
        return;
    }
    const int64_t f = a.first_out;
    const int words = ctx->words();
    if (mvs_launch_expand_geom(&ctx->sc, r, &a, s) != 0) throw Fail{MVS_E_HIP, "expand_geom launch failed"};
    score_device(ctx, a.n, r.c + 3 * f, r.R + f, wid, a.thr, r.xy + 2 * f, r.mask + words * f, r.count + f,
                 nullptr, s);
    if (mvs_launch_expand_accept(r, &a, s) != 0) throw Fail{MVS_E_HIP, "expand_accept launch failed"};
}

// CellTable.filter_out_outlier (MVS2.py:132-158) over n accepted patches in
// fill order (patch e: cell = which_cell of its projection, V-list mask,
// |V| = count, avg_ncc_score, centre, normal).  Q_table[(v, ci, cj)] holds
// patch e |V| times for every v of its V list at its one cell (every V entry
// carries the same projection, MVS2.py:105-107); keys are visited in
// (v, ci, cj) order; threshold = sum of (1 - avg) over the key's current
// list / its length (a filled cell whose list emptied raises
// ZeroDivisionError, MVS2.py:144 -> MVS_E_DIVZERO); a patch p2 of the list
// is an outlier if |V2| avg2 < threshold and some other patch p1 of the list
// is not its neighbour (is_patch_neighbor, 0.2, MVS2.py:298-299); outliers
// leave every key (|V|^2 "remove a outlier" lines each).  alive[e] = 0 for
// the removed.
void filter_outliers_core(int64_t n, int words, int nci, int ncj, const int32_t* cell, const uint64_t* mask,
                          const int32_t* count, const double* avg, const double* c, const double* nrm,
                          uint8_t* alive, int64_t* removed_out, int64_t* lines_out) {
    // (key, patch) entries, key = (v * nci + ci) * ncj + cj; patches in fill order
    std::vector<std::pair<int64_t, int32_t>> ent;
    for (int64_t e = 0; e < n; ++e) {
        alive[e] = 1;
        const int cx = cell[2 * e], cy = cell[2 * e + 1];
        if (cx < 0 || cx >= nci || cy < 0 || cy >= ncj) continue;
        for (int w = 0; w < words; ++w)
            for (uint64_t m = mask[e * words + w]; m; m &= m - 1) {
                const int v = 64 * w + __builtin_ctzll(m);
                ent.push_back({((int64_t)v * nci + cx) * ncj + cy, (int32_t)e});
            }
    }
    std::sort(ent.begin(), ent.end());
    // is_patch_neighbor(p1, p2, 0.2) (MVS2.py:298-299), numpy's 3-element dots
    auto neighbor = [&](int32_t e1, int32_t e2) {
        const double* c1 = &c[3 * (int64_t)e1];
        const double* c2 = &c[3 * (int64_t)e2];
        const double* n1 = &nrm[3 * (int64_t)e1];
        const double* n2 = &nrm[3 * (int64_t)e2];
        const double d0 = c1[0] - c2[0], d1 = c1[1] - c2[1], d2 = c1[2] - c2[2];
        return std::fabs(fma_dot3(d0, d1, d2, n1[0], n1[1], n1[2]) + fma_dot3(d0, d1, d2, n2[0], n2[1], n2[2])) < 0.2;
    };
    std::vector<int32_t> L, out;
    int64_t removed = 0, lines = 0;
    for (size_t b = 0; b < ent.size();) {
        size_t e_end = b;
        while (e_end < ent.size() && ent[e_end].first == ent[b].first) ++e_end;
        L.clear();
        double thr = 0.0;
        int64_t len = 0;
        for (size_t k = b; k < e_end; ++k) {
            const int32_t e = ent[k].second;
            if (!alive[e]) continue;
            L.push_back(e);
            const int m = count[e];
            for (int i = 0; i < m; ++i) thr += 1.0 - avg[e];
            len += m;
        }
        if (len == 0) {
            const int64_t key = ent[b].first;
            char msg[200];
            std::snprintf(msg, sizeof msg,
                          "filter_out_outlier: ZeroDivisionError (MVS2.py:144): every patch of filled cell "
                          "(view %lld, %lld, %lld) was removed before it was visited",
                          (long long)(key / ((int64_t)nci * ncj)), (long long)(key / ncj % nci),
                          (long long)(key % ncj));
            throw Fail{MVS_E_DIVZERO, msg};
        }
        thr /= (double)len;
        out.clear();
        for (int32_t p2 : L) {
            if (!((double)count[p2] * avg[p2] < thr)) continue;
            for (int32_t p1 : L)
                if (p1 != p2 && !neighbor(p1, p2)) {
                    out.push_back(p2);
                    break;
                }
        }
        for (int32_t p : out)
            if (alive[p]) {
                alive[p] = 0;
                ++removed;
                lines += (int64_t)count[p] * count[p];
            }
        b = e_end;
    }
    *removed_out = removed;
    *lines_out = lines;
}

// ---------------------------------------------------------------------------
// Stage engine: seeding + ordered expansion commit
// ---------------------------------------------------------------------------

struct Engine {
    mvs_ctx* ctx;
    int V, words, cs, wid, vlb;
    int flags = 0;   // mvs_stage_set_options at the stage's start
    double scale;
    int nci, ncj;
    int64_t max_pops;
    hipStream_t s;

    // record table (device) + host mirror
    DevBuf<double> d_c, d_n, d_xy;
    DevBuf<uint64_t> d_mask;
    DevBuf<int32_t> d_R, d_count, d_cell;
    DevBuf<uint8_t> d_color, d_accept;
    DevBuf<ChildJob> d_jobs;
    int64_t nrec = 0, cap = 0;
    std::vector<uint64_t> h_mask;
    std::vector<int32_t> h_count, h_cell;
    std::vector<uint8_t> h_accept, h_enq;
    std::vector<int64_t> h_child;   // first child record, -1 = unscored

    std::vector<uint64_t> table;    // [nci][ncj][words] view bitmasks, 1 = vacant (CellTable)
    std::vector<int32_t> events;    // accepted patch objects, in fill order
    int64_t n_accepted = -1;        // events before filter_outliers (-1: not filtered)
    int64_t n_seeds = 0;
    int64_t stat_tests = 0, stat_scored = 0, stat_sweeps = 0, stat_seed_cands = 0;

    RecordsDev recs() {
        RecordsDev r;
        r.c = d_c.p; r.n = d_n.p; r.xy = d_xy.p; r.mask = d_mask.p; r.R = d_R.p;
        r.count = d_count.p; r.color = d_color.p; r.accept = d_accept.p; r.cell = d_cell.p;
        return r;
    }

    void reserve(int64_t need) {
        if (need <= cap) return;
        int64_t nc = std::max<int64_t>(need, std::max<int64_t>(cap * 2, 1 << 16));
        d_c.grow(nc * 3, nrec * 3, s);
        d_n.grow(nc * 3, nrec * 3, s);
        d_xy.grow(nc * 2, nrec * 2, s);
        d_mask.grow(nc * words, nrec * words, s);
        d_R.grow(nc, nrec, s);
        d_count.grow(nc, nrec, s);
        d_cell.grow(nc * 2, nrec * 2, s);
        d_color.grow(nc * 4, nrec * 4, s);
        d_accept.grow(nc, nrec, s);
        cap = nc;
        h_mask.resize(nc * words);
        h_count.resize(nc);
        h_cell.resize(nc * 2);
        h_accept.resize(nc);
        h_enq.resize(nc);
        h_child.resize(nc, -1);
    }

    bool vacant(int v, long ci, long cj) const {
        if (ci >= nci || ci < 0) return false;
        if (cj >= ncj || cj < 0) return false;
        return (table[((int64_t)ci * ncj + cj) * words + (v >> 6)] >> (v & 63)) & 1u;
    }

    // CellTable.fill_with_point for every V entry of record r (MVS2.py:98-107,
    // 258-259, 401-402); the Q-table side is reconstructed from `events`.
    void fill_record(int64_t r) {
        // every V entry carries the same projection, so one cell gets the
        // record's whole view mask: clear those views' vacancy bits at once
        const int cx = h_cell[2 * r], cy = h_cell[2 * r + 1];
        if (cx < 0 || cx >= nci || cy < 0 || cy >= ncj) return;
        uint64_t* cell = &table[((int64_t)cx * ncj + cy) * words];
        for (int w = 0; w < words; ++w) cell[w] &= ~h_mask[r * words + w];
    }

    void fetch_range(int64_t first, int64_t n) {
        if (n == 0) return;
        HIPCHK(hipMemcpyAsync(h_mask.data() + first * words, d_mask.p + first * words,
                              n * words * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(h_count.data() + first, d_count.p + first, n * sizeof(int32_t),
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(h_cell.data() + 2 * first, d_cell.p + 2 * first,
                              2 * n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(h_accept.data() + first, d_accept.p + first, n * sizeof(uint8_t),
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }

    // ---- seeding: MVS2.py:205-260 ----
    void seed(int64_t n_tracks, const int64_t* off, const int32_t* ov, const float* oxy) {
        const std::vector<CamDev>& cams = ctx->cams;
        struct Cand {
            double key[5];
            double c[3], n[3];
            uint8_t color[3];
            int R;
        };
        std::vector<std::vector<Cand>> per_track(n_tracks);
        const int H = ctx->H, W = ctx->W;
        for (int64_t tr = 0; tr < n_tracks; ++tr) {
            const int64_t o0 = off[tr], o1 = off[tr + 1];
            if (o1 - o0 < 1) continue;
            const int Rr = ov[o0];
            if (Rr < 0 || Rr >= V) throw Fail{MVS_E_ARG, "track view index out of range"};
            const double base[2] = {(double)oxy[2 * o0], (double)oxy[2 * o0 + 1]};
            const double* O = cams[Rr].O;
            for (int64_t o = o0 + 1; o < o1; ++o) {
                const int k = ov[o];
                if (k < 0 || k >= V) throw Fail{MVS_E_ARG, "track view index out of range"};
                double P1[12], P2[12];
                // getProjectionMatrix = K @ [r|t] (utils.py:234-236)
                for (int rr = 0; rr < 3; ++rr)
                    for (int cc = 0; cc < 4; ++cc) {
                        const CamDev& a = cams[Rr];
                        const CamDev& b = cams[k];
                        auto e = [&](const CamDev& m, int q) { return cc < 3 ? m.R[3 * q + cc] : m.t[q]; };
                        P1[rr * 4 + cc] = fma_dot3(kmat(Rr, rr, 0), kmat(Rr, rr, 1), kmat(Rr, rr, 2),
                                                   e(a, 0), e(a, 1), e(a, 2));
                        P2[rr * 4 + cc] = fma_dot3(kmat(k, rr, 0), kmat(k, rr, 1), kmat(k, rr, 2),
                                                   e(b, 0), e(b, 1), e(b, 2));
                    }
                const double pt[2] = {(double)oxy[2 * o], (double)oxy[2 * o + 1]};
                double X4[4];
                triangulate(P1, P2, base, pt, X4);
                Cand cd;
                for (int q = 0; q < 3; ++q) cd.c[q] = X4[3] == 0 ? 0 * X4[q] : X4[q] / X4[3];
                const double d0 = cd.c[0] - O[0], d1 = cd.c[1] - O[1], d2 = cd.c[2] - O[2];
                const double dist = std::sqrt((d0 * d0 + d1 * d1) + d2 * d2);
                for (int q = 0; q < 3; ++q) cd.n[q] = (O[q] - cd.c[q]) / dist;
                // get_color(imgs[k], x, y) = img[int(y)][int(x)] (MVS2.py:248)
                const long xi = (long)oxy[2 * o], yi = (long)oxy[2 * o + 1];
                const int yy = py_wrap(yi, H), xx = py_wrap(xi, W);
                if (yy < 0 || yy >= H || xx < 0 || xx >= W) throw Fail{MVS_E_ARG, "observation outside image"};
                const uint8_t* px = ctx->h_rgb.data() + (((int64_t)k * H + yy) * W + xx) * 3;
                cd.color[0] = px[0]; cd.color[1] = px[1]; cd.color[2] = px[2];
                cd.R = Rr;
                cd.key[0] = dist; cd.key[1] = cd.c[0]; cd.key[2] = cd.c[1]; cd.key[3] = cd.c[2];
                cd.key[4] = Rr;
                per_track[tr].push_back(cd);
            }
            // MyPatchHeapSort pops in increasing (dist, c0, c1, c2, R) (MVS2.py:13-31)
            std::stable_sort(per_track[tr].begin(), per_track[tr].end(), [](const Cand& a, const Cand& b) {
                for (int q = 0; q < 5; ++q) {
                    if (a.key[q] < b.key[q]) return true;
                    if (a.key[q] > b.key[q]) return false;
                }
                return false;
            });
        }
        // score every seed candidate in one batch (thr 0.4, MVS2.py:255)
        std::vector<double> hc;
        std::vector<int32_t> hr;
        for (auto& v : per_track)
            for (auto& cd : v) {
                hc.insert(hc.end(), cd.c, cd.c + 3);
                hr.push_back(cd.R);
            }
        const int64_t nc = (int64_t)hr.size();
        stat_seed_cands = nc;
        DevBuf<double> dc, dxy, davg;
        DevBuf<int32_t> dr, dcount;
        DevBuf<uint64_t> dmask;
        dc.alloc(nc * 3); dxy.alloc(nc * 2); davg.alloc(nc); dr.alloc(nc); dcount.alloc(nc);
        dmask.alloc(nc * words);
        std::vector<double> xy(nc * 2);
        std::vector<uint64_t> mask(nc * words);
        std::vector<int32_t> count(nc);
        if (nc) {
            HIPCHK(hipMemcpyAsync(dc.p, hc.data(), nc * 3 * sizeof(double), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(dr.p, hr.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, s));
            score_device(ctx, nc, dc.p, dr.p, wid, 0.4, dxy.p, dmask.p, dcount.p, davg.p, s);
            HIPCHK(hipMemcpyAsync(xy.data(), dxy.p, nc * 2 * sizeof(double), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(mask.data(), dmask.p, nc * words * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(count.data(), dcount.p, nc * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        stat_scored += nc;
        // first candidate (heap order) with |V| >= vlb is the track's patch
        std::vector<double> rc, rn, rxy;
        std::vector<uint8_t> rcol;
        std::vector<int32_t> rR, rcount, rcell;
        std::vector<uint64_t> rmask;
        int64_t idx = 0;
        for (auto& v : per_track) {
            int64_t first = idx;
            idx += (int64_t)v.size();
            for (size_t q = 0; q < v.size(); ++q) {
                const int64_t i = first + (int64_t)q;
                stat_tests++;
                if (count[i] >= vlb) {
                    const Cand& cd = v[q];
                    rc.insert(rc.end(), cd.c, cd.c + 3);
                    rn.insert(rn.end(), cd.n, cd.n + 3);
                    rxy.insert(rxy.end(), &xy[2 * i], &xy[2 * i] + 2);
                    rcol.insert(rcol.end(), {cd.color[0], cd.color[1], cd.color[2], 0});
                    rR.push_back(cd.R);
                    rcount.push_back(count[i]);
                    rmask.insert(rmask.end(), &mask[i * words], &mask[i * words] + words);
                    rcell.push_back((int32_t)std::floor(xy[2 * i] / cs));
                    rcell.push_back((int32_t)std::floor(xy[2 * i + 1] / cs));
                    break;
                }
            }
        }
        n_seeds = (int64_t)rR.size();
        reserve(std::max<int64_t>(n_seeds, 1));
        if (n_seeds) {
            std::vector<uint8_t> acc(n_seeds, 1);
            HIPCHK(hipMemcpyAsync(d_c.p, rc.data(), n_seeds * 3 * sizeof(double), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_n.p, rn.data(), n_seeds * 3 * sizeof(double), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_xy.p, rxy.data(), n_seeds * 2 * sizeof(double), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_mask.p, rmask.data(), n_seeds * words * sizeof(uint64_t), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_R.p, rR.data(), n_seeds * sizeof(int32_t), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_count.p, rcount.data(), n_seeds * sizeof(int32_t), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_cell.p, rcell.data(), n_seeds * 2 * sizeof(int32_t), hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_color.p, rcol.data(), n_seeds * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d_accept.p, acc.data(), n_seeds, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
            std::copy(rmask.begin(), rmask.end(), h_mask.begin());
            std::copy(rcount.begin(), rcount.end(), h_count.begin());
            std::copy(rcell.begin(), rcell.end(), h_cell.begin());
            std::fill(h_accept.begin(), h_accept.begin() + n_seeds, 1);
        }
        nrec = n_seeds;
        for (int64_t r = 0; r < n_seeds; ++r) {
            fill_record(r);
            events.push_back((int32_t)r);
        }
    }

    double kmat(int v, int r, int c) const { return ctx->K[9 * v + 3 * r + c]; }

    // ---- patch_expansion: MVS2.py:308-404 ----
    // The FIFO loop is split into steps so that several GPUs can share a
    // sweep: plan() commits in reference order until the FIFO head needs
    // children nobody has scored yet and lays out the next sweep's jobs;
    // score_range() scores a contiguous slice of them into the record table;
    // fetch_sweep() brings the sweep's gates to the host for the next plan().
    // Every rank runs the same plan() on the same records, so all commits
    // agree.
    // the FIFO, run-length encoded: an accepted patch is enqueued |V| times in
    // a row (MVS2.py:376-379), stored once with its copy count
    struct QEntry {
        int32_t rec;
        int32_t left;
    };
    std::vector<QEntry> queue;
    int64_t queued = 0;              // copies still in the FIFO
    size_t qhead = 0;
    std::vector<int32_t> unscored;   // records in order of first enqueue
    size_t ucur = 0;
    int64_t pops = 0;
    std::vector<ChildJob> jobs;
    int64_t sweep_first = 0, sweep_n = 0;
    bool trace = false;

    void expand_init() {
        trace = std::getenv("MVS_TRACE") != nullptr;
        queue.clear();
        queue.reserve(1 << 18);
        queued = 0;
        qhead = 0;
        unscored.clear();
        ucur = 0;
        pops = 0;
        for (int64_t r = 0; r < n_seeds; ++r) {
            queue.push_back(QEntry{(int32_t)r, 1});
            ++queued;
            unscored.push_back((int32_t)r);
            h_enq[r] = 1;
        }
    }

    // Commit, then plan the next sweep; returns its job count (0: stage finished).
    int64_t plan() {
        // ordered commit until the FIFO head has no scored children
        while (qhead < queue.size() && pops < max_pops) {
            const int32_t r = queue[qhead].rec;
            const int64_t base = h_child[r];
            if (base < 0) break;
            // the FIFO is known ahead: pull the records a few entries on, and
            // the children of the entries nearer, into cache (the record
            // arrays outgrow the caches; the walk is latency-bound)
            if (qhead + 8 < queue.size()) {
                const int32_t r8 = queue[qhead + 8].rec;
                __builtin_prefetch(&h_child[r8]);
                __builtin_prefetch(&h_cell[2 * (int64_t)r8]);
                __builtin_prefetch(&h_mask[(int64_t)r8 * words]);
            }
            if (qhead + 3 < queue.size()) {
                const int64_t b3 = h_child[queue[qhead + 3].rec];
                if (b3 >= 0) {
                    __builtin_prefetch(&h_accept[b3]);
                    __builtin_prefetch(&h_count[b3]);
                }
            }
            if (--queue[qhead].left == 0) ++qhead;
            --queued;
            ++pops;
            const long ci = h_cell[2 * r], cj = h_cell[2 * r + 1];
            // every view of the parent tests the same four cells (ci +- 1, cj +- 1):
            // their vacancy words are loaded once per mask word and again after
            // a fill (is_vacant, MVS2.py:90-96; off-grid cells are never vacant)
            const uint64_t* nb4[4];
            for (int k = 0; k < 4; ++k) {
                const long a = ci + ((k >> 1) ? 1 : -1), bb = cj + ((k & 1) ? 1 : -1);
                nb4[k] = (a < 0 || a >= nci || bb < 0 || bb >= ncj) ? nullptr : &table[(a * ncj + bb) * words];
            }
            int h = 0;
            for (int w = 0; w < words; ++w) {
                uint64_t vw[4];
                auto load4 = [&]() {
                    for (int k = 0; k < 4; ++k) vw[k] = nb4[k] ? nb4[k][w] : 0ull;
                };
                load4();
                uint64_t m = h_mask[(int64_t)r * words + w];
                while (m) {
                    const int v = 64 * w + __builtin_ctzll(m);
                    const uint64_t bit = m & (~m + 1);
                    m &= m - 1;
                    for (int i = -1; i <= 1; i += 2) {
                        const int64_t child = base + 2 * h + (i > 0 ? 1 : 0);
                        for (int j = -1; j <= 1; j += 2) {
                            if (!(vw[(i > 0 ? 2 : 0) + (j > 0 ? 1 : 0)] & bit)) continue;
                            ++stat_tests;
                            if (trace) std::fprintf(stderr, "E pop %lld rec %d v %d i %d j %d child %lld acc %d cnt %d cell %d %d\n",
                                (long long)pops, r, v, i, j, (long long)child, (int)h_accept[child], h_count[child], h_cell[2*child], h_cell[2*child+1]);
                            if (h_accept[child]) {
                                fill_record(child);
                                load4();
                                events.push_back((int32_t)child);
                                if (h_count[child] > 0) {
                                    queue.push_back(QEntry{(int32_t)child, h_count[child]});
                                    queued += h_count[child];
                                }
                                if (!h_enq[child]) {
                                    h_enq[child] = 1;
                                    unscored.push_back((int32_t)child);
                                }
                                break;
                            }
                        }
                    }
                    ++h;
                }
            }
        }
        if (qhead >= queue.size() || pops >= max_pops) {
            stat_pops = pops;
            stat_queue_left = queued;
            sweep_n = 0;
            return 0;
        }
        // sweep: the children of the next unscored records (first-enqueue order)
        const int64_t remaining = max_pops - pops;
        int64_t want = std::min<int64_t>(std::max<int64_t>(remaining / 4, 2048), 262144);
        want = std::min<int64_t>(want, (int64_t)(unscored.size() - ucur));
        jobs.clear();
        sweep_first = nrec;
        for (int64_t k = 0; k < want; ++k) {
            const int32_t r = unscored[ucur + k];
            h_child[r] = sweep_first + (int64_t)jobs.size();
            for (int w = 0; w < words; ++w) {
                uint64_t m = h_mask[(int64_t)r * words + w];
                while (m) {
                    const int v = 64 * w + __builtin_ctzll(m);
                    m &= m - 1;
                    jobs.push_back(ChildJob{r, (int16_t)v, (int16_t)-1});
                    jobs.push_back(ChildJob{r, (int16_t)v, (int16_t)1});
                }
            }
        }
        ucur += want;
        sweep_n = (int64_t)jobs.size();
        reserve(nrec + sweep_n);
        d_jobs.ensure(sweep_n);
        if (sweep_n)
            HIPCHK(hipMemcpyAsync(d_jobs.p, jobs.data(), sweep_n * sizeof(ChildJob), hipMemcpyHostToDevice, s));
        nrec += sweep_n;
        stat_scored += sweep_n;
        stat_sweeps++;
        return sweep_n;
    }

    ExpandArgs sweep_args(int64_t b, int64_t e) {
        ExpandArgs a{};
        a.n = e - b;
        a.first_out = sweep_first + b;
        a.jobs = d_jobs.p + b;
        a.cell_size = cs;
        a.vlb = vlb;
        a.dist_thr = 0.05 / scale;
        a.thr = 0.7;
        a.exact_hits = ctx->d_exact.p;
        return a;
    }

    // k_expand over jobs [b, e) of the planned sweep -> records sweep_first + [b, e)
    void score_range(int64_t b, int64_t e) {
        if (e <= b) return;
        expand_device(ctx, recs(), sweep_args(b, e), wid, s);
    }

    // Multi-GPU sweep, one rank's share: the geometry (centre, normal,
    // projection, colour, cell) of EVERY child of the sweep -- it depends only
    // on parent records every rank holds -- and the photo test + accept test of
    // the rank's own slice [b, e).  The other ranks then need only the slices'
    // masks (mvs_stage_ingest -> ingest_masks).
    void score_range_sharded(int64_t b, int64_t e) {
        const ExpandArgs all = sweep_args(0, sweep_n);
        if (sweep_n > 0 && mvs_launch_expand_geom(&ctx->sc, recs(), &all, s) != 0)
            throw Fail{MVS_E_HIP, "expand_geom launch failed"};
        if (e <= b) return;
        const ExpandArgs a = sweep_args(b, e);
        const int64_t f = a.first_out;
        RecordsDev r = recs();
        score_device(ctx, a.n, r.c + 3 * f, r.R + f, wid, a.thr, r.xy + 2 * f, r.mask + words * f,
                     r.count + f, nullptr, s);
        if (mvs_launch_expand_accept(r, &a, s) != 0) throw Fail{MVS_E_HIP, "expand_accept launch failed"};
    }

    // another rank's slice [b, e): its masks (words per child, from the
    // all-gathered buffer) into the record table, then count and accept
    void ingest_masks(int64_t b, int64_t e, const int64_t* d_masks) {
        if (e <= b) return;
        HIPCHK(hipMemcpyAsync(d_mask.p + (sweep_first + b) * words, d_masks, (e - b) * words * sizeof(uint64_t),
                              hipMemcpyDeviceToDevice, s));
        const ExpandArgs a = sweep_args(b, e);
        if (mvs_launch_expand_ingest(recs(), &a, words, s) != 0) throw Fail{MVS_E_HIP, "expand_ingest launch failed"};
    }

    void fetch_sweep() { fetch_range(sweep_first, sweep_n); }

    // host time per phase (seconds), printed by mvs_stage_run under MVS_STAGE_TIMES
    double t_plan = 0, t_score = 0, t_fetch = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }

    void expand() {
        expand_init();
        for (;;) {
            double t0 = now();
            const int64_t nj = plan();
            double t1 = now();
            t_plan += t1 - t0;
            if (nj == 0) break;
            score_range(0, sweep_n);
            HIPCHK(hipStreamSynchronize(s));
            double t2 = now();
            t_score += t2 - t1;
            fetch_sweep();
            t_fetch += now() - t2;
        }
    }

    // contiguous slice of n jobs for `rank` (sizes differ by <= 1; parallel.shard_range)
    static void shard(int64_t n, int rank, int world, int64_t* b, int64_t* e) {
        const int64_t base = n / world, extra = n % world;
        *b = rank * base + std::min<int64_t>(rank, extra);
        *e = *b + base + (rank < extra ? 1 : 0);
    }
    int64_t stat_pops = 0, stat_queue_left = 0;

    // reconstruct_from_Q order (MVS2.py:159-173): key (view, ci, cj)
    // lexicographic, append order within a key, first sight of each object.  A
    // patch is appended under (u, cell) for every u in its V list, so its first
    // sight is at (min u, cell), in fill order among equal keys: a stable sort
    // of the acceptance events by (min view, cell x, cell y).  All on the
    // device: event keys (k_event_keys), a stable LSD radix sort (hipCUB) and
    // the row gather (k_gather_rows) into the result's HBM rows.
    double t_out[5] = {0, 0, 0, 0, 0};   // upload, keys + sort, rows, -, end stamp (MVS_STAGE_TIMES)
    DevBuf<int32_t> o_ev, o_vals, o_init;

    // CellTable.filter_out_outlier (MVS2.py:132-158) as if MVS2.py:281 ran it,
    // between the expansion and reconstruct_from_Q.  Q_table[(v, ci, cj)] holds
    // every accepted patch whose V list contains v, at the cell of its
    // projection, |V| times (fill_with_point appends it once per V entry, and
    // every V entry carries the same projection).  Keys are visited in
    // (v, ci, cj) order; for each, threshold = sum(1 - avg) over the current
    // list / its length, and a patch p2 of the list is an outlier if
    // |V2|·avg2 < threshold and some other patch p1 of the list is not its
    // neighbour (is_patch_neighbor, 0.2); outliers leave every key they are in
    // (printing "remove a outlier" per entry: |V|² per patch).  avg_ncc_score
    // is recomputed in the reference's arithmetic first (k_exact_avg).
    // Patches leave whole, so the output order of the rest is unchanged.
    void filter_outliers(mvs_stage_result* res) {
        const int64_t nev = (int64_t)events.size();
        n_accepted = nev;
        if (nev == 0) return;
        // avg_ncc_score per event, c and n per record
        DevBuf<int32_t> d_ids;
        DevBuf<double> d_avg;
        d_ids.alloc(nev);
        d_avg.alloc(nev);
        HIPCHK(hipMemcpyAsync(d_ids.p, events.data(), nev * sizeof(int32_t), hipMemcpyHostToDevice, s));
        if (mvs_launch_exact_avg(&ctx->sc, recs(), wid, d_ids.p, nev, d_avg.p, s) != 0)
            throw Fail{MVS_E_HIP, "exact_avg launch failed"};
        std::vector<double> avg(nev), hc(nrec * 3), hn(nrec * 3);
        HIPCHK(hipMemcpyAsync(avg.data(), d_avg.p, nev * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(hc.data(), d_c.p, nrec * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(hn.data(), d_n.p, nrec * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        // the events' patches, in fill order
        std::vector<int32_t> ecell(2 * nev), ecount(nev);
        std::vector<uint64_t> emask(nev * words);
        std::vector<double> ec(3 * nev), en(3 * nev);
        for (int64_t e = 0; e < nev; ++e) {
            const int64_t r = events[e];
            ecell[2 * e] = h_cell[2 * r];
            ecell[2 * e + 1] = h_cell[2 * r + 1];
            ecount[e] = h_count[r];
            for (int w = 0; w < words; ++w) emask[e * words + w] = h_mask[r * words + w];
            for (int j = 0; j < 3; ++j) {
                ec[3 * e + j] = hc[3 * r + j];
                en[3 * e + j] = hn[3 * r + j];
            }
        }
        std::vector<uint8_t> alive(nev, 1);
        int64_t removed = 0, lines = 0;
        filter_outliers_core(nev, words, nci, ncj, ecell.data(), emask.data(), ecount.data(), avg.data(),
                             ec.data(), en.data(), alive.data(), &removed, &lines);
        std::vector<int32_t> kept;
        kept.reserve(nev - removed);
        for (int64_t e = 0; e < nev; ++e)
            if (alive[e]) kept.push_back(events[e]);
        events.swap(kept);
        res->filt[0] = removed;
        res->filt[1] = lines;
    }
    DevBuf<uint64_t> o_keys, o_keys_s;
    DevBuf<uint8_t> o_tmp;

    void output(mvs_stage_result* res) {
        double ta = now();
        const int64_t nev = (int64_t)events.size();
        res->device = ctx->device;
        res->n_init = n_seeds;
        res->d_init.alloc((size_t)std::max<int64_t>(n_seeds, 1) * 6);
        if (n_seeds) {
            o_init.ensure(n_seeds);
            std::vector<int32_t> ids(n_seeds);
            for (int64_t r = 0; r < n_seeds; ++r) ids[r] = (int32_t)r;
            HIPCHK(hipMemcpyAsync(o_init.p, ids.data(), n_seeds * sizeof(int32_t), hipMemcpyHostToDevice, s));
            if (mvs_launch_gather_rows(recs(), o_init.p, n_seeds, res->d_init.p, s) != 0)
                throw Fail{MVS_E_HIP, "gather_rows launch failed"};
            HIPCHK(hipStreamSynchronize(s));   // ids leaves scope
        }
        res->d_all.alloc((size_t)std::max<int64_t>(nev, 1) * 6);
        if (nev) {
            o_ev.ensure(nev);
            o_vals.ensure(nev);
            o_keys.ensure(nev);
            o_keys_s.ensure(nev);
            HIPCHK(hipMemcpyAsync(o_ev.p, events.data(), nev * sizeof(int32_t), hipMemcpyHostToDevice, s));
            double tb = now();
            t_out[0] = tb - ta;
            if (mvs_launch_event_keys(recs(), words, o_ev.p, nev, nci, ncj, o_keys.p, s) != 0)
                throw Fail{MVS_E_HIP, "event_keys launch failed"};
            const uint64_t kmax = (uint64_t)V * nci * ncj;   // keys < kmax; never-emitted events: ~0
            int bits = 1;
            while (bits < 63 && (1ull << bits) <= kmax) ++bits;
            size_t tmp_bytes = 0;
            if (mvs_sort_pairs(nullptr, &tmp_bytes, o_keys.p, o_keys_s.p, o_ev.p, o_vals.p, nev, bits, s) != 0)
                throw Fail{MVS_E_HIP, "sort sizing failed"};
            o_tmp.ensure(tmp_bytes);
            if (mvs_sort_pairs(o_tmp.p, &tmp_bytes, o_keys.p, o_keys_s.p, o_ev.p, o_vals.p, nev, bits, s) != 0)
                throw Fail{MVS_E_HIP, "sort failed"};
            // emitted events = keys below kmax; the never-emitted (~0) sort last
            uint64_t last = 0;
            HIPCHK(hipMemcpyAsync(&last, o_keys_s.p + nev - 1, sizeof last, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            int64_t n_all = nev;
            if (last >= kmax) {
                std::vector<uint64_t> ks(nev);
                HIPCHK(hipMemcpy(ks.data(), o_keys_s.p, nev * sizeof(uint64_t), hipMemcpyDeviceToHost));
                n_all = std::lower_bound(ks.begin(), ks.end(), kmax) - ks.begin();
            }
            double tc = now();
            t_out[1] = tc - tb;
            res->n_all = n_all;
            if (mvs_launch_gather_rows(recs(), o_vals.p, n_all, res->d_all.p, s) != 0)
                throw Fail{MVS_E_HIP, "gather_rows launch failed"};
            HIPCHK(hipStreamSynchronize(s));
            t_out[2] = now() - tc;
        }
        res->stats[0] = stat_pops;
        res->stats[1] = stat_tests;
        res->stats[2] = n_accepted >= 0 ? n_accepted : (int64_t)events.size();
        res->stats[3] = stat_queue_left;
        res->stats[4] = stat_scored;
        res->stats[5] = stat_sweeps;
        res->stats[6] = stat_seed_cands;
    }
};

}  // namespace

struct mvs_stage {
    mvs_ctx* ctx = nullptr;
    std::unique_ptr<Engine> E;
    int rank = 0, world = 1;
    int stage_state = 0;   // 0 planned nothing, 1 sweep planned, 2 slice scored, 3 finished
};

namespace {
Engine* make_engine(mvs_ctx* ctx, int cell_size, double scale, int wid, int64_t max_pops) {
    std::unique_ptr<Engine> E(new Engine());
    E->ctx = ctx;
    E->V = ctx->V;
    E->words = ctx->words();
    E->cs = cell_size;
    E->wid = wid;
    E->vlb = ctx->V > 2 ? 3 : 2;   // MVS2.py:200-203
    E->scale = scale;
    // CellTable: ceil((W-1)/cs) x ceil((H-1)/cs) per view (MVS2.py:88)
    E->nci = (int)std::ceil((double)(ctx->W - 1) / cell_size);
    E->ncj = (int)std::ceil((double)(ctx->H - 1) / cell_size);
    E->max_pops = std::min<int64_t>(std::max<int64_t>(max_pops, 0), 100000);   // MVS2.py:321
    E->s = ctx->stream;
    // the stage's options are fixed when it starts (mvs_stage_set_options
    // between mvs_stage_begin and mvs_stage_finish does not change it)
    E->flags = ctx->stage_flags;
    // CellTable as vacancy bitmasks, one per cell: bit v of cell (ci, cj) = 1
    // while view v's cell is vacant (np.ones, MVS2.py:88)
    E->table.assign((size_t)E->nci * E->ncj * E->words, 0);
    for (int64_t k = 0; k < (int64_t)E->nci * E->ncj; ++k)
        for (int w = 0; w < E->words; ++w) {
            const int nv = std::min(64, ctx->V - 64 * w);
            E->table[k * E->words + w] = nv >= 64 ? ~0ull : ((1ull << nv) - 1ull);
        }
    return E.release();
}

void finish_engine(mvs_ctx* ctx, Engine* E, mvs_stage_result* res) {
    // the exact-path counter first: a device-to-host copy issued after
    // output() has written ~35 MB of fresh host memory took ~25 ms here
    int32_t h = 0;
    HIPCHK(hipMemcpyAsync(&h, ctx->d_exact.p, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    const double t = Engine::now();
    if (E->flags & MVS_STAGE_FILTER_OUTLIERS) E->filter_outliers(res);
    E->output(res);
    E->t_out[4] = Engine::now() - t;
    res->stats[7] = h;
}
}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------

extern "C" {

const char* mvs_version(void) { return "mvs_amd 0.1 (gfx950)"; }

const char* mvs_last_error(const mvs_ctx* ctx) {
    return ctx ? ctx->err.c_str() : g_err.c_str();
}

int mvs_ctx_create(int device, int V, int H, int W, const uint8_t* rgb, const double* K,
                   const double* R, const double* t, const double* Rp, mvs_ctx** out) {
    if (!out || !rgb || !K || !R || !t) return set_err(nullptr, Fail{MVS_E_ARG, "null argument"});
    *out = nullptr;
    if (V < 1 || V > MVS_MAX_VIEWS || H < 16 || W < 16 || H > 65536 || W > 65536)
        return set_err(nullptr, Fail{MVS_E_UNSUPPORTED, "need 1 <= V <= 256 and 16 <= H, W <= 65536"});
    std::unique_ptr<mvs_ctx> ctx(new mvs_ctx());
    ctx->device = device;
    int rc = guarded(ctx.get(), [&]() {
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw Fail{MVS_E_ARG, "no such HIP device"};
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->V = V; ctx->H = H; ctx->W = W;
        ctx->Wq = (W + 3) / 4 + 1;   // +1 zero quad: the last aligned dword read of a row
        const int64_t npx = (int64_t)V * H * W;
        ctx->h_rgb.assign(rgb, rgb + npx * 3);
        ctx->d_rgb.alloc(npx * 3);
        HIPCHK(hipMemcpyAsync(ctx->d_rgb.p, rgb, npx * 3, hipMemcpyHostToDevice, ctx->stream));
        const int64_t stack_bytes = (int64_t)H * ctx->Wq * V * 4;
        ctx->d_stack.alloc(stack_bytes + 64);
        HIPCHK(hipMemsetAsync(ctx->d_stack.p, 0, stack_bytes + 64, ctx->stream));
        // view-major copy: 8 zero bytes left of column 0, >= 24 right of W-1,
        // pitch a multiple of 16 (SceneDev)
        ctx->sc.Wp = (W + 32 + 15) & ~15;
        const int64_t gv_bytes = (int64_t)V * H * ctx->sc.Wp + 64;
        ctx->d_gv.alloc(gv_bytes);
        HIPCHK(hipMemsetAsync(ctx->d_gv.p, 0, gv_bytes, ctx->stream));
        ctx->sc.V = V; ctx->sc.H = H; ctx->sc.W = W; ctx->sc.Wq = ctx->Wq;
        ctx->sc.row_bytes = (int64_t)ctx->Wq * V * 4;
        ctx->sc.stack = ctx->d_stack.p;
        ctx->sc.rgb = ctx->d_rgb.p;
        ctx->sc.gv = ctx->d_gv.p + 8;
        if (mvs_launch_build_scene(&ctx->sc, ctx->d_rgb.p, ctx->d_stack.p, ctx->d_gv.p, ctx->stream) != 0)
            throw Fail{MVS_E_HIP, "build_scene launch failed"};
        build_cameras(ctx.get(), K, R, t, Rp);
        ctx->K.assign(K, K + 9 * V);
        ctx->d_cams.alloc(V);
        HIPCHK(hipMemcpyAsync(ctx->d_cams.p, ctx->cams.data(), V * sizeof(CamDev), hipMemcpyHostToDevice, ctx->stream));
        ctx->d_exact.alloc(1);
        HIPCHK(hipMemsetAsync(ctx->d_exact.p, 0, sizeof(int32_t), ctx->stream));
        ctx->d_stats.alloc(4);
        HIPCHK(hipMemsetAsync(ctx->d_stats.p, 0, 4 * sizeof(unsigned long long), ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        ctx->sc.cams = ctx->d_cams.p;
        if (const char* km = std::getenv("MVS_SCORE_KERNEL")) {
            if (!std::strcmp(km, "direct")) ctx->kernel_mode = 1;
            else if (!std::strcmp(km, "tiled")) ctx->kernel_mode = 2;
            else if (!std::strcmp(km, "mma")) ctx->tab_mode = 1;   // tiled, in-kernel moments
            else if (!std::strcmp(km, "tab")) ctx->tab_mode = 2;   // tiled, tables at every V
        }
        if (const char* sw = std::getenv("MVS_SCORER_WGS")) ctx->scorer_wgs = std::max(0, std::atoi(sw));
        if (const char* tl = std::getenv("MVS_TAB_LIMIT")) ctx->tab_limit = std::max<int64_t>(1, std::atoll(tl));
        return 0;
    });
    if (rc != 0) {
        g_err = ctx->err;
        return rc;
    }
    *out = ctx.release();
    return 0;
}

void mvs_ctx_destroy(mvs_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // the scratch's last users may be any streams (some perhaps destroyed by now)
    if (ctx->scratch_order.used || ctx->pack_order.used) (void)hipDeviceSynchronize();
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    for (hipEvent_t e : ctx->ev) (void)hipEventDestroy(e);
    if (ctx->scratch_order.ev) (void)hipEventDestroy(ctx->scratch_order.ev);
    if (ctx->pack_order.ev) (void)hipEventDestroy(ctx->pack_order.ev);
    delete ctx;
}

int mvs_kernel_timing(mvs_ctx* ctx, int enable) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    return guarded(ctx, [&]() {
        if (enable < 0) throw Fail{MVS_E_ARG, "timing period must be >= 0"};
        ctx->timing = enable != 0;
        if (ctx->timing) {
            ctx->ev_used = 0;   // disabling keeps the record readable
            ctx->timing_period = enable;
            ctx->timing_count = 0;
        }
        return 0;
    });
}

int mvs_kernel_time(mvs_ctx* ctx, double* total_ms, int64_t* launches) {
    if (!ctx || !total_ms || !launches) return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    return guarded(ctx, [&]() {
        double tot = 0.0;
        for (size_t k = 0; k + 1 < ctx->ev_used; k += 2) {
            HIPCHK(hipEventSynchronize(ctx->ev[k + 1]));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, ctx->ev[k], ctx->ev[k + 1]));
            tot += ms;
        }
        *total_ms = tot;
        *launches = (int64_t)(ctx->ev_used / 2);
        return 0;
    });
}

const char* mvs_timed_kernel(const mvs_ctx* ctx) { return ctx ? ctx->timed_name : ""; }

int mvs_ctx_rebuild(mvs_ctx* ctx, void* stream) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    return guarded(ctx, [&]() {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        if (mvs_launch_build_scene(&ctx->sc, ctx->d_rgb.p, ctx->d_stack.p, ctx->d_gv.p, s) != 0)
            throw Fail{MVS_E_HIP, "build_scene launch failed"};
        // the window-moment tables built so far follow the scene
        for (int w = 1; w <= MVS_MAX_WID; ++w)
            if (ctx->mom_ok[w]) {
                const MomentsDev m = ctx->moments(w);
                if (mvs_launch_moments(&ctx->sc, &m, s) != 0) throw Fail{MVS_E_HIP, "moments launch failed"};
            }
        return 0;
    });
}

int mvs_ctx_rproj(const mvs_ctx* ctx, double* Rp) {
    if (!ctx || !Rp) return MVS_E_ARG;
    for (int v = 0; v < ctx->V; ++v) std::memcpy(Rp + 9 * v, ctx->cams[v].Rp, 9 * sizeof(double));
    return 0;
}

int mvs_score_device(mvs_ctx* ctx, int64_t n, const double* d_c, const int32_t* d_ref, int wid,
                     double min_ncc, double* d_xy, uint64_t* d_mask, int32_t* d_count,
                     double* d_avg, void* stream) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (n < 0) return set_err(ctx, Fail{MVS_E_ARG, "n < 0"});
    if (n > 0 && (!d_c || !d_ref || !d_xy || !d_mask || !d_count))
        return set_err(ctx, Fail{MVS_E_ARG, "null device pointer"});
    return guarded(ctx, [&]() {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        score_device(ctx, n, d_c, d_ref, wid, min_ncc, d_xy, d_mask, d_count, d_avg, s);
        return 0;
    });
}

int mvs_score_device_rec(mvs_ctx* ctx, int64_t n, const double* d_c, const int32_t* d_ref, int wid,
                         double min_ncc, double* d_xy, int64_t* d_rec, void* stream) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (n < 0 || (n > 0 && (!d_c || !d_ref || !d_xy || !d_rec)) || ((uintptr_t)d_rec & 15) != 0)
        return set_err(ctx, Fail{MVS_E_ARG, "bad arguments (records must be 16-B aligned)"});
    return guarded(ctx, [&]() {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        score_device(ctx, n, d_c, d_ref, wid, min_ncc, d_xy, (uint64_t*)d_rec, nullptr, nullptr, s);
        return 0;
    });
}

int mvs_filter_outliers(int64_t n, int words, int nci, int ncj, const int32_t* cell, const uint64_t* mask,
                        const int32_t* count, const double* avg, const double* c, const double* nrm,
                        uint8_t* alive, int64_t* stats) {
    if (n < 0 || words < 1 || nci < 1 || ncj < 1 || !stats ||
        (n > 0 && (!cell || !mask || !count || !avg || !c || !nrm || !alive)))
        return set_err(nullptr, Fail{MVS_E_ARG, "bad arguments"});
    return guarded(nullptr, [&]() {
        filter_outliers_core(n, words, nci, ncj, cell, mask, count, avg, c, nrm, alive, &stats[0], &stats[1]);
        return 0;
    });
}

int mvs_pack_accepted(mvs_ctx* ctx, int64_t n, int64_t offset, const int32_t* d_count, const uint64_t* d_mask,
                      const double* d_c, int vlb, int64_t cap, int64_t* d_out, void* stream) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (n < 0 || cap < 0 || !d_out || (n > 0 && !d_mask))
        return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    return guarded(ctx, [&]() {
        hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
        // the pack's own scratch (counter, ticket): ordered against the
        // previous pack only, so that a pack on a communication stream does
        // not order the next sweep's scoring behind it
        ctx->pack_order.acquire(s);
        if (!ctx->p_ctl.p) {
            ctx->p_ctl.ensure(32);
            HIPCHK(hipMemsetAsync(ctx->p_ctl.p, 0, 32 * sizeof(unsigned long long), s));
        }
        if (mvs_launch_pack_accepted(n, offset, d_count, d_mask, d_c, ctx->words(), vlb, cap, ctx->p_ctl.p, d_out,
                                     s) != 0)
            throw Fail{MVS_E_HIP, "pack launch failed"};
        ctx->pack_order.release(s);
        return 0;
    });
}

int mvs_proxy_copy(void* d_dst, const void* d_src, int64_t bytes, int workgroups, void* stream) {
    if (bytes < 0 || (bytes % 16) != 0 || workgroups < 1 || (bytes > 0 && (!d_dst || !d_src)))
        return set_err(nullptr, Fail{MVS_E_ARG, "bad arguments"});
    if (mvs_launch_proxy_copy(d_dst, d_src, bytes, workgroups, (hipStream_t)stream) != 0)
        return set_err(nullptr, Fail{MVS_E_HIP, "proxy copy launch failed"});
    return 0;
}

int mvs_set_scorer_grid(mvs_ctx* ctx, int workgroups) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (workgroups < 0) return set_err(ctx, Fail{MVS_E_ARG, "workgroups must be >= 0"});
    ctx->scorer_wgs = workgroups;
    return 0;
}

int mvs_score(mvs_ctx* ctx, int64_t n, const double* c, const int32_t* ref, int wid, double min_ncc,
              double* xy, uint64_t* mask, int32_t* count, double* avg) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (n < 0 || (n > 0 && (!c || !ref || !xy || !mask || !count || !avg)))
        return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    return guarded(ctx, [&]() {
        for (int64_t i = 0; i < n; ++i)
            if (ref[i] < 0 || ref[i] >= ctx->V) throw Fail{MVS_E_ARG, "ref view out of range"};
        if (n == 0) return 0;
        hipStream_t s = ctx->stream;
        const int words = ctx->words();
        ctx->s_c.ensure(n * 3); ctx->s_ref.ensure(n); ctx->s_xy.ensure(n * 2);
        ctx->s_mask.ensure(n * words); ctx->s_count.ensure(n); ctx->s_avg.ensure(n);
        HIPCHK(hipMemcpyAsync(ctx->s_c.p, c, n * 3 * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(ctx->s_ref.p, ref, n * sizeof(int32_t), hipMemcpyHostToDevice, s));
        score_device(ctx, n, ctx->s_c.p, ctx->s_ref.p, wid, min_ncc, ctx->s_xy.p, ctx->s_mask.p,
                     ctx->s_count.p, ctx->s_avg.p, s);
        HIPCHK(hipMemcpyAsync(xy, ctx->s_xy.p, n * 2 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(mask, ctx->s_mask.p, n * words * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(count, ctx->s_count.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(avg, ctx->s_avg.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        return 0;
    });
}

int64_t mvs_exact_hits(mvs_ctx* ctx) {
    if (!ctx) return MVS_E_ARG;
    int32_t h = 0;
    int rc = guarded(ctx, [&]() {
        HIPCHK(hipMemcpyAsync(&h, ctx->d_exact.p, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        return 0;
    });
    return rc ? rc : h;
}

int mvs_stream_retiring(mvs_ctx* ctx, void* stream) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (!stream) return 0;   // the library's own stream is never retired by a caller
    return guarded(ctx, [&]() {
        ctx->scratch_order.retire((hipStream_t)stream);
        ctx->pack_order.retire((hipStream_t)stream);
        return 0;
    });
}

int mvs_scorer_stats(mvs_ctx* ctx, int64_t* out) {
    if (!ctx || !out) return set_err(ctx, Fail{MVS_E_ARG, "null argument"});
    return guarded(ctx, [&]() {
        unsigned long long h[4] = {0, 0, 0, 0};
        HIPCHK(hipMemcpyAsync(h, ctx->d_stats.p, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        for (int k = 0; k < 3; ++k) out[k] = (int64_t)h[k];
        return 0;
    });
}

int mvs_ncc_windows(int64_t n, int npx, const uint8_t* d_a, const uint8_t* d_b, double thr,
                    int force_exact, double* d_ncc, uint8_t* d_pass, void* stream) {
    if (npx < 1 || npx > 128) return set_err(nullptr, Fail{MVS_E_UNSUPPORTED, "npx must be in 1..128"});
    int rc = mvs_launch_ncc_windows(n, npx, d_a, d_b, thr, force_exact, d_ncc, d_pass, (hipStream_t)stream);
    if (rc) return set_err(nullptr, Fail{MVS_E_HIP, "ncc_windows launch failed"});
    return 0;
}

int mvs_stage_run(mvs_ctx* ctx, int64_t n_tracks, const int64_t* track_off, const int32_t* obs_view,
                  const float* obs_xy, int cell_size, double scale, int wid, int64_t max_pops,
                  mvs_stage_result** out) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (!out || n_tracks < 0 || (n_tracks > 0 && (!track_off || !obs_view || !obs_xy)) || cell_size < 1)
        return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    if (wid != 3 && wid != 5) return set_err(ctx, Fail{MVS_E_UNSUPPORTED, "stage supports wid 3 or 5"});
    *out = nullptr;
    return guarded(ctx, [&]() {
        std::unique_ptr<mvs_stage_result> res(new mvs_stage_result());
        std::unique_ptr<Engine> E(make_engine(ctx, cell_size, scale, wid, max_pops));
        HIPCHK(hipMemsetAsync(ctx->d_exact.p, 0, sizeof(int32_t), ctx->stream));
        const double t0 = Engine::now();
        E->seed(n_tracks, track_off, obs_view, obs_xy);
        const double t1 = Engine::now();
        E->expand();
        const double t2 = Engine::now();
        finish_engine(ctx, E.get(), res.get());
        const double t3 = Engine::now();
        res->times[0] = t1 - t0;
        res->times[1] = E->t_plan;
        res->times[2] = E->t_score;
        res->times[3] = E->t_fetch;
        res->times[4] = t3 - t2;
        res->times[5] = t3 - t0;
        if (std::getenv("MVS_STAGE_TIMES"))
            std::fprintf(stderr, "stage times: seed %.4f s, expand %.4f s (commit/plan %.4f, GPU sweeps %.4f, "
                                 "fetch %.4f), output %.4f s\n",
                         t1 - t0, t2 - t1, E->t_plan, E->t_score, E->t_fetch, t3 - t2);
        if (std::getenv("MVS_STAGE_TIMES"))
            std::fprintf(stderr, "  output: events upload %.4f, keys + sort %.4f, row gather %.4f s; output() %.4f s\n",
                         E->t_out[0], E->t_out[1], E->t_out[2], E->t_out[4]);
        *out = res.release();
        if (std::getenv("MVS_STAGE_TIMES")) {
            const double td = Engine::now();
            E.reset();
            std::fprintf(stderr, "  engine teardown %.4f s\n", Engine::now() - td);
        }
        return 0;
    });
}

int mvs_stage_begin(mvs_ctx* ctx, int64_t n_tracks, const int64_t* track_off, const int32_t* obs_view,
                    const float* obs_xy, int cell_size, double scale, int wid, int64_t max_pops,
                    int rank, int world, mvs_stage** out) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (!out || n_tracks < 0 || (n_tracks > 0 && (!track_off || !obs_view || !obs_xy)) || cell_size < 1 ||
        world < 1 || rank < 0 || rank >= world)
        return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    if (wid != 3 && wid != 5) return set_err(ctx, Fail{MVS_E_UNSUPPORTED, "stage supports wid 3 or 5"});
    *out = nullptr;
    return guarded(ctx, [&]() {
        std::unique_ptr<mvs_stage> st(new mvs_stage());
        st->ctx = ctx;
        st->rank = rank;
        st->world = world;
        st->E.reset(make_engine(ctx, cell_size, scale, wid, max_pops));
        HIPCHK(hipMemsetAsync(ctx->d_exact.p, 0, sizeof(int32_t), ctx->stream));
        // seeding is replicated: every rank scores the (small) seed batch itself
        st->E->seed(n_tracks, track_off, obs_view, obs_xy);
        st->E->expand_init();
        *out = st.release();
        return 0;
    });
}

int64_t mvs_stage_plan(mvs_stage* st) {
    if (!st) return set_err(nullptr, Fail{MVS_E_ARG, "null stage"});
    if (st->stage_state == 1 || st->stage_state == 2)
        return set_err(st->ctx, Fail{MVS_E_ARG, "mvs_stage_plan: previous sweep not ingested"});
    if (st->stage_state == 3) return 0;
    int64_t nj = 0;
    const int rc = guarded(st->ctx, [&]() {
        nj = st->E->plan();
        return 0;
    });
    if (rc) return rc;
    st->stage_state = nj > 0 ? 1 : 3;
    return nj;
}

int mvs_stage_record_width(const mvs_stage* st) {
    if (!st) return MVS_E_ARG;
    return st->E->words;
}

int mvs_stage_score_slice(mvs_stage* st, int64_t* d_out) {
    if (!st) return set_err(nullptr, Fail{MVS_E_ARG, "null stage"});
    if (st->stage_state != 1) return set_err(st->ctx, Fail{MVS_E_ARG, "mvs_stage_score_slice: no planned sweep"});
    if (st->world > 1 && !d_out) return set_err(st->ctx, Fail{MVS_E_ARG, "null slice buffer"});
    const int rc = guarded(st->ctx, [&]() {
        Engine* E = st->E.get();
        if (st->world == 1) {
            E->score_range(0, E->sweep_n);
        } else {
            int64_t b, e;
            Engine::shard(E->sweep_n, st->rank, st->world, &b, &e);
            E->score_range_sharded(b, e);
            // the slice's exchange record is its mask words: contiguous in the table
            if (e > b)
                HIPCHK(hipMemcpyAsync(d_out, E->d_mask.p + (E->sweep_first + b) * E->words,
                                      (e - b) * E->words * sizeof(uint64_t), hipMemcpyDeviceToDevice, E->s));
        }
        HIPCHK(hipStreamSynchronize(E->s));
        return 0;
    });
    if (rc == 0) st->stage_state = 2;
    return rc;
}

int mvs_stage_ingest(mvs_stage* st, const int64_t* d_all) {
    if (!st) return set_err(nullptr, Fail{MVS_E_ARG, "null stage"});
    if (st->stage_state != 2) return set_err(st->ctx, Fail{MVS_E_ARG, "mvs_stage_ingest: slice not scored"});
    if (st->world > 1 && !d_all) return set_err(st->ctx, Fail{MVS_E_ARG, "null gathered buffer"});
    const int rc = guarded(st->ctx, [&]() {
        Engine* E = st->E.get();
        if (st->world > 1) {
            const int64_t smax = (E->sweep_n + st->world - 1) / st->world;
            const int64_t w = E->words;
            for (int r = 0; r < st->world; ++r) {
                if (r == st->rank) continue;   // own slice is already in the record table
                int64_t b, e;
                Engine::shard(E->sweep_n, r, st->world, &b, &e);
                E->ingest_masks(b, e, d_all + (int64_t)r * smax * w);
            }
        }
        E->fetch_sweep();
        return 0;
    });
    if (rc == 0) st->stage_state = 0;
    return rc;
}

int mvs_stage_finish(mvs_stage* st, mvs_stage_result** out) {
    if (!st || !out) return set_err(st ? st->ctx : nullptr, Fail{MVS_E_ARG, "bad arguments"});
    if (st->stage_state != 3) return set_err(st->ctx, Fail{MVS_E_ARG, "mvs_stage_finish: stage not finished"});
    *out = nullptr;
    return guarded(st->ctx, [&]() {
        std::unique_ptr<mvs_stage_result> res(new mvs_stage_result());
        finish_engine(st->ctx, st->E.get(), res.get());
        *out = res.release();
        return 0;
    });
}

void mvs_stage_destroy(mvs_stage* st) {
    if (!st) return;
    if (st->ctx) (void)hipSetDevice(st->ctx->device);
    delete st;
}

int64_t mvs_stage_count(const mvs_stage_result* res, int which) {
    if (!res) return MVS_E_ARG;
    return which ? res->n_all : res->n_init;
}

int mvs_stage_rows(const mvs_stage_result* res, int which, double* rows) {
    if (!res || !rows) return MVS_E_ARG;
    const int64_t n = which ? res->n_all : res->n_init;
    if (n == 0) return 0;
    if (hipSetDevice(res->device) != hipSuccess ||
        hipMemcpy(rows, which ? res->d_all.p : res->d_init.p, n * 6 * sizeof(double), hipMemcpyDeviceToHost) !=
            hipSuccess)
        return set_err(nullptr, Fail{MVS_E_HIP, "rows copy failed"});
    return 0;
}

int mvs_stage_rows_device(const mvs_stage_result* res, int which, double* d_rows, void* stream) {
    if (!res || !d_rows) return MVS_E_ARG;
    const int64_t n = which ? res->n_all : res->n_init;
    if (n == 0) return 0;
    if (hipSetDevice(res->device) != hipSuccess ||
        hipMemcpyAsync(d_rows, which ? res->d_all.p : res->d_init.p, n * 6 * sizeof(double),
                       hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess)
        return set_err(nullptr, Fail{MVS_E_HIP, "rows copy failed"});
    return 0;
}

int mvs_stage_stats(const mvs_stage_result* res, int64_t* stats) {
    if (!res || !stats) return MVS_E_ARG;
    std::memcpy(stats, res->stats, sizeof res->stats);
    return 0;
}

int mvs_stage_times(const mvs_stage_result* res, double* times) {
    if (!res || !times) return MVS_E_ARG;
    std::memcpy(times, res->times, 6 * sizeof(double));
    return 0;
}

int mvs_exact_avg(mvs_ctx* ctx, int64_t n, const int32_t* ref, const double* xy, const uint64_t* mask, int wid,
                  double* avg) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (n < 0 || (n > 0 && (!ref || !xy || !mask || !avg))) return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    if (wid != 3 && wid != 5) return set_err(ctx, Fail{MVS_E_UNSUPPORTED, "exact avg supports wid 3 or 5"});
    return guarded(ctx, [&]() {
        const int words = ctx->words();
        for (int64_t i = 0; i < n; ++i) {
            if (ref[i] < 0 || ref[i] >= ctx->V) throw Fail{MVS_E_ARG, "ref view out of range"};
            // a V list names other views (MVS2.py:66-67) inside the scene; a
            // non-empty one needs a valid window (HarrisFeatures.py:128)
            bool any = false;
            for (int w = 0; w < words; ++w) {
                uint64_t m = mask[i * words + w];
                const int nv = ctx->V - 64 * w;
                if (nv < 64 && (m >> nv)) throw Fail{MVS_E_ARG, "mask names a view >= V"};
                if (ref[i] / 64 == w && ((m >> (ref[i] % 64)) & 1ull))
                    throw Fail{MVS_E_ARG, "mask names the reference view itself"};
                any |= m != 0;
            }
            if (any) {
                const double x = xy[2 * i], y = xy[2 * i + 1];
                if (!(x > -1e9 && x < 1e9 && y > -1e9 && y < 1e9)) throw Fail{MVS_E_ARG, "non-finite projection"};
                const int q = (int)x, r = (int)y;
                if (!(r - wid >= 0 && r + wid + 1 < ctx->H && q - wid > 0 && q + wid + 1 < ctx->W))
                    throw Fail{MVS_E_ARG, "mask bits set for a window outside the image"};
            }
        }
        if (n == 0) return 0;
        hipStream_t s = ctx->stream;
        ctx->s_ref.ensure(n); ctx->s_xy.ensure(n * 2); ctx->s_mask.ensure(n * words); ctx->s_avg.ensure(n);
        HIPCHK(hipMemcpyAsync(ctx->s_ref.p, ref, n * sizeof(int32_t), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(ctx->s_xy.p, xy, n * 2 * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(ctx->s_mask.p, mask, n * words * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        RecordsDev rec{};
        rec.R = ctx->s_ref.p;
        rec.xy = ctx->s_xy.p;
        rec.mask = ctx->s_mask.p;
        if (mvs_launch_exact_avg(&ctx->sc, rec, wid, nullptr, n, ctx->s_avg.p, s) != 0)
            throw Fail{MVS_E_HIP, "exact_avg launch failed"};
        HIPCHK(hipMemcpyAsync(avg, ctx->s_avg.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        return 0;
    });
}

int mvs_stage_set_options(mvs_ctx* ctx, int flags) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (flags & ~MVS_STAGE_FILTER_OUTLIERS) return set_err(ctx, Fail{MVS_E_ARG, "unknown stage option"});
    ctx->stage_flags = flags;
    return 0;
}

int mvs_stage_filter_stats(const mvs_stage_result* res, int64_t* out) {
    if (!res || !out) return MVS_E_ARG;
    out[0] = res->filt[0];
    out[1] = res->filt[1];
    return 0;
}

void mvs_stage_free(mvs_stage_result* res) {
    if (!res) return;
    (void)hipSetDevice(res->device);
    delete res;
}

int mvs_expand_candidates(mvs_ctx* ctx, int64_t n_parents, const double* pc, const double* pn,
                          const double* pxy, int64_t n_jobs, const int32_t* job_parent,
                          const int32_t* job_view, const int32_t* job_di, int cell_size,
                          double scale, int wid, double min_ncc, double* X, double* nX,
                          uint8_t* color, double* xy, uint64_t* mask, int32_t* count,
                          uint8_t* accept) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    if (n_parents < 0 || n_jobs < 0 || cell_size < 1) return set_err(ctx, Fail{MVS_E_ARG, "bad arguments"});
    if (wid != 3 && wid != 5) return set_err(ctx, Fail{MVS_E_UNSUPPORTED, "expand supports wid 3 or 5"});
    return guarded(ctx, [&]() {
        for (int64_t k = 0; k < n_jobs; ++k)
            if (job_parent[k] < 0 || job_parent[k] >= n_parents || job_view[k] < 0 ||
                job_view[k] >= ctx->V || (job_di[k] != 1 && job_di[k] != -1))
                throw Fail{MVS_E_ARG, "bad job"};
        if (n_jobs == 0) return 0;
        hipStream_t s = ctx->stream;
        const int words = ctx->words();
        const int64_t nr = n_parents + n_jobs;
        DevBuf<double> c_, n_, xy_;
        DevBuf<uint64_t> m_;
        DevBuf<int32_t> R_, cnt_, cell_;
        DevBuf<uint8_t> col_, acc_;
        DevBuf<ChildJob> jobs_;
        c_.alloc(nr * 3); n_.alloc(nr * 3); xy_.alloc(nr * 2); m_.alloc(nr * words); R_.alloc(nr);
        cnt_.alloc(nr); cell_.alloc(nr * 2); col_.alloc(nr * 4); acc_.alloc(nr); jobs_.alloc(n_jobs);
        std::vector<ChildJob> jobs(n_jobs);
        for (int64_t k = 0; k < n_jobs; ++k)
            jobs[k] = ChildJob{job_parent[k], (int16_t)job_view[k], (int16_t)job_di[k]};
        HIPCHK(hipMemcpyAsync(c_.p, pc, n_parents * 3 * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(n_.p, pn, n_parents * 3 * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(xy_.p, pxy, n_parents * 2 * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(jobs_.p, jobs.data(), n_jobs * sizeof(ChildJob), hipMemcpyHostToDevice, s));
        RecordsDev r;
        r.c = c_.p; r.n = n_.p; r.xy = xy_.p; r.mask = m_.p; r.R = R_.p; r.count = cnt_.p;
        r.color = col_.p; r.accept = acc_.p; r.cell = cell_.p;
        ExpandArgs a{};
        a.n = n_jobs;
        a.first_out = n_parents;
        a.jobs = jobs_.p;
        a.cell_size = cell_size;
        a.vlb = ctx->V > 2 ? 3 : 2;
        a.dist_thr = 0.05 / scale;
        a.thr = min_ncc;
        a.exact_hits = ctx->d_exact.p;
        expand_device(ctx, r, a, wid, s);
        std::vector<uint8_t> col4(n_jobs * 4);
        HIPCHK(hipMemcpyAsync(X, c_.p + n_parents * 3, n_jobs * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(nX, n_.p + n_parents * 3, n_jobs * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(xy, xy_.p + n_parents * 2, n_jobs * 2 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(mask, m_.p + n_parents * words, n_jobs * words * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(count, cnt_.p + n_parents, n_jobs * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(accept, acc_.p + n_parents, n_jobs, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(col4.data(), col_.p + n_parents * 4, n_jobs * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int64_t k = 0; k < n_jobs; ++k)
            for (int q = 0; q < 3; ++q) color[3 * k + q] = col4[4 * k + q];
        return 0;
    });
}

int mvs_rodrigues_roundtrip(const double* R, double* Rp) {
    if (!R || !Rp) return MVS_E_ARG;
    rodrigues_roundtrip(R, Rp);
    return 0;
}

int mvs_triangulate(const double* P1, const double* P2, const double* x1, const double* x2, double* X4) {
    if (!P1 || !P2 || !x1 || !x2 || !X4) return MVS_E_ARG;
    triangulate(P1, P2, x1, x2, X4);
    return 0;
}

// ---- SfM front-end (HarrisFeatures.py, SFM.py) ----

int mvs_harris_points(mvs_ctx* ctx, int view, int32_t* out, int64_t cap, int64_t* n_out) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    return guarded(ctx, [&]() -> int {
        if (!n_out || (cap > 0 && !out)) throw Fail{MVS_E_ARG, "null output"};
        if (view < 0 || view >= ctx->V) throw Fail{MVS_E_ARG, "view out of range"};
        // BORDER_REFLECT_101 of a 3x3 Sobel needs two pixels per axis
        if (ctx->H < 2 || ctx->W < 2) throw Fail{MVS_E_UNSUPPORTED, "Harris needs images of at least 2x2"};
        const int64_t npx = (int64_t)ctx->H * ctx->W;
        ctx->f_resp.ensure(npx);
        ctx->f_dil.ensure(npx);
        ctx->f_key.ensure(1);
        ctx->f_rows.ensure(2 * (size_t)ctx->H + 1);
        hipStream_t s = ctx->stream;
        int32_t* rowcnt = ctx->f_rows.p;
        int32_t* rowoff = ctx->f_rows.p + ctx->H;
        if (mvs_launch_harris(&ctx->sc, view, 0.04, ctx->f_resp.p, ctx->f_dil.p, ctx->f_key.p, rowcnt,
                              rowoff, s) != 0)
            throw Fail{MVS_E_HIP, "harris launch failed"};
        int32_t total = 0;
        HIPCHK(hipMemcpyAsync(&total, rowoff + ctx->H, sizeof total, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        *n_out = total;
        const int64_t m = std::min<int64_t>(total, cap);
        if (m > 0) {
            ctx->f_pts.ensure(2 * (size_t)total);
            if (mvs_launch_harris_write(&ctx->sc, ctx->f_dil.p, ctx->f_key.p, rowoff, ctx->f_pts.p, total,
                                        s) != 0)
                throw Fail{MVS_E_HIP, "harris write launch failed"};
            HIPCHK(hipMemcpyAsync(out, ctx->f_pts.p, 2 * m * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        return 0;
    });
}

int mvs_match_two_sided(mvs_ctx* ctx, int view_a, const int32_t* pts_a, int64_t n_a, int view_b,
                        const int32_t* pts_b, int64_t n_b, int wid, double thr, int32_t* m12,
                        int32_t* best12, int32_t* best21) {
    if (!ctx) return set_err(nullptr, Fail{MVS_E_ARG, "null context"});
    return guarded(ctx, [&]() -> int {
        if (n_a < 0 || n_b < 0 || (n_a && (!pts_a || !m12)) || (n_b && !pts_b))
            throw Fail{MVS_E_ARG, "bad point arrays"};
        if (view_a < 0 || view_a >= ctx->V || view_b < 0 || view_b >= ctx->V)
            throw Fail{MVS_E_ARG, "view out of range"};
        if (wid < 1 || (2 * wid + 1) * (2 * wid + 1) > 128) throw Fail{MVS_E_UNSUPPORTED, "wid must be 1..5"};
        // getDescFeatures keeps only windows inside these bounds (HarrisFeatures.py:128)
        for (int side = 0; side < 2; ++side) {
            const int32_t* p = side ? pts_b : pts_a;
            const int64_t n = side ? n_b : n_a;
            for (int64_t i = 0; i < n; ++i) {
                const int r = p[2 * i], c = p[2 * i + 1];
                if (!(r - wid >= 0 && r + wid + 1 < ctx->H && c - wid > 0 && c + wid + 1 < ctx->W))
                    throw Fail{MVS_E_ARG, "point outside getDescFeatures' bounds"};
            }
        }
        if (n_a == 0) return 0;
        const int npx = (2 * wid + 1) * (2 * wid + 1);
        constexpr int DW = 32;   // descriptor dwords (kDescWords)
        const int64_t n = n_a + n_b;
        ctx->f_pts.ensure(2 * (size_t)n);
        ctx->f_desc.ensure((size_t)DW * n + 4);
        ctx->f_mom.ensure(2 * (size_t)n);
        ctx->f_best.ensure((size_t)n);
        hipStream_t s = ctx->stream;
        HIPCHK(hipMemcpyAsync(ctx->f_pts.p, pts_a, 2 * n_a * sizeof(int32_t), hipMemcpyHostToDevice, s));
        if (n_b)
            HIPCHK(hipMemcpyAsync(ctx->f_pts.p + 2 * n_a, pts_b, 2 * n_b * sizeof(int32_t),
                                  hipMemcpyHostToDevice, s));
        uint32_t* dA = ctx->f_desc.p;
        uint32_t* dB = ctx->f_desc.p + (size_t)DW * n_a;
        int32_t* S = ctx->f_mom.p;
        int32_t* SS = ctx->f_mom.p + n;
        if (mvs_launch_gather_desc(&ctx->sc, view_a, ctx->f_pts.p, n_a, wid, dA, S, SS, s) != 0 ||
            mvs_launch_gather_desc(&ctx->sc, view_b, ctx->f_pts.p + 2 * n_a, n_b, wid, dB, S + n_a,
                                   SS + n_a, s) != 0)
            throw Fail{MVS_E_HIP, "descriptor launch failed"};
        int32_t* b12 = ctx->f_best.p;
        int32_t* b21 = ctx->f_best.p + n_a;
        if (mvs_launch_match_rows(dA, S, SS, n_a, dB, S + n_a, SS + n_a, n_b, npx, thr, b12, s) != 0 ||
            mvs_launch_match_rows(dB, S + n_a, SS + n_a, n_b, dA, S, SS, n_a, npx, thr, b21, s) != 0)
            throw Fail{MVS_E_HIP, "match launch failed"};
        std::vector<int32_t> h12(n_a), h21(n_b);
        HIPCHK(hipMemcpyAsync(h12.data(), b12, n_a * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        if (n_b) HIPCHK(hipMemcpyAsync(h21.data(), b21, n_b * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        // MatchTwoSided's symmetric check (HarrisFeatures.py:60-64)
        for (int64_t i = 0; i < n_a; ++i) {
            const int32_t j = h12[i];
            m12[i] = (j >= 0 && h21[j] == (int32_t)i) ? j : -1;
        }
        if (best12) std::copy(h12.begin(), h12.end(), best12);
        if (best21) std::copy(h21.begin(), h21.end(), best21);
        return 0;
    });
}

int mvs_sfm_pair(const double* KA, const double* RA, const double* tA, const double* KB,
                 const double* RB, const double* tB, int64_t n, const float* q, const float* tr,
                 double max_err, float* pt, uint8_t* keep) {
    if (!KA || !RA || !tA || !KB || !RB || !tB || n < 0 || (n && (!q || !tr || !pt || !keep)))
        return set_err(nullptr, Fail{MVS_E_ARG, "null argument"});
    double P1[12], P2[12], RpA[9], RpB[9];
    projection_matrix(KA, RA, tA, P1);
    projection_matrix(KB, RB, tB, P2);
    rodrigues_roundtrip(RA, RpA);
    rodrigues_roundtrip(RB, RpB);
    for (int64_t i = 0; i < n; ++i) {
        // cv2.triangulatePoints on float32 points: double DLT, float32 result
        const double x1[2] = {q[2 * i], q[2 * i + 1]}, x2[2] = {tr[2 * i], tr[2 * i + 1]};
        double X4[4];
        triangulate(P1, P2, x1, x2, X4);
        const float w = (float)X4[3];
        keep[i] = 0;
        pt[3 * i] = pt[3 * i + 1] = pt[3 * i + 2] = 0.f;
        if (w == 0.f) continue;                    // SFM.py:69-72: not added
        float p[3];
        for (int k = 0; k < 3; ++k) p[k] = (float)X4[k] / w;
        for (int k = 0; k < 3; ++k) pt[3 * i + k] = p[k];
        // projectPoint on the float32 point: double projection, float32 result;
        // np.linalg.norm of the float32 residual (SFM.py:75-78)
        const double M[3] = {p[0], p[1], p[2]};
        double oa[2], ob[2];
        project_host(KA, RpA, tA, M, oa);
        project_host(KB, RpB, tB, M, ob);
        const float ra0 = (float)oa[0] - q[2 * i], ra1 = (float)oa[1] - q[2 * i + 1];
        const float rb0 = (float)ob[0] - tr[2 * i], rb1 = (float)ob[1] - tr[2 * i + 1];
        const float ea = std::sqrt(ra0 * ra0 + ra1 * ra1), eb = std::sqrt(rb0 * rb0 + rb1 * rb1);
        keep[i] = ((double)ea > max_err || (double)eb > max_err) ? 0 : 1;
    }
    return 0;
}

}  // extern "C"

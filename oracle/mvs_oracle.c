/*
 * mvs_oracle.c -- CPU restatement of the reference MVS hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product package may link, load or
 * call this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the CPU baseline.
 *
 * Reference: MarvinChung/simple-implementation-of-structure-from-motion-and-
 * multi-view-stereo-by-python (read-only copy at /root/reference).
 * Every function cites the reference lines it restates.  Floating-point
 * operation order follows what numpy 2.2 + OpenBLAS 0.3.29 execute for the
 * reference's Python expressions (measured in this container, see DESIGN.md
 * "FP op order"): 3-element np.dot / 3x3 matvec = FMA chain
 *   fma(a2,b2, fma(a1,b1, a0*b0)),
 * np.sum over float64 = numpy pairwise sum (8 accumulators for n <= 128),
 * Python float arithmetic = plain IEEE binary64.  Compile with
 * -ffp-contract=off so no other product gets fused.
 *
 * Third-party arithmetic restated here (OpenCV is absent from the image, so
 * these restatements are what the golden fixtures were generated with; parity
 * against real OpenCV is UNPINNED, version unknown -- the reference pins
 * none):
 *   cv2.cvtColor(BGR2GRAY, 8u)   -> or_gray_from_rgb      (HarrisFeatures.py:125)
 *   cv2.Rodrigues (both ways)     -> or_rodrigues_*        (utils.py:242)
 *   cv2.projectPoints (no dist.)  -> or_project            (utils.py:243)
 *   cv2.triangulatePoints         -> or_triangulate        (utils.py:239)
 *   cv::JacobiSVD (used by both)  -> or_jacobi_svd
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_MAXV 1024

/* ------------------------------------------------------------------------ */
/* OpenCV restatements                                                      */
/* ------------------------------------------------------------------------ */

/* cv2.cvtColor(img, COLOR_BGR2GRAY) on an 8u image (HarrisFeatures.py:125).
 * OpenCV fixed point (yuv_shift 14): gray = (B*1868 + G*9617 + R*4899 + 8192)>>14
 * with B = channel 0.  The reference feeds RGB data (main.py:18), so channel 0
 * is red and gets the blue weight. */
void or_gray_from_rgb(const uint8_t *rgb, int64_t npix, uint8_t *gray) {
    for (int64_t i = 0; i < npix; ++i) {
        const uint8_t *p = rgb + 3 * i;
        gray[i] = (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14);
    }
}

/* cv::JacobiSVDImpl_<double> (one-sided Jacobi on the rows of At, n rows of
 * length m), eps = 10*DBL_EPSILON, minval = DBL_MIN, as called by
 * cv::SVD::compute for a square matrix (At = A^T on entry, U^T on exit). */
void or_jacobi_svd(double *At, double *Wout, double *Vt, int m, int n) {
    double W[16];
    const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
    int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = hypot(p, beta), c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0; Aj[k] = t1;
                    a += t0 * t0; b += t1 * t1;
                }
                W[i] = a; W[j] = b;
                changed = 1;
                double *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (int k = 0; k < n; k++) {
                    double t0 = c * Vi[k] + s * Vj[k];
                    double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0; Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++) if (W[j] < W[k]) j = k;
        if (i != j) {
            double tw = W[i]; W[i] = W[j]; W[j] = tw;
            for (int k = 0; k < m; k++) { double t = At[i * m + k]; At[i * m + k] = At[j * m + k]; At[j * m + k] = t; }
            for (int k = 0; k < n; k++) { double t = Vt[i * n + k]; Vt[i * n + k] = Vt[j * n + k]; Vt[j * n + k] = t; }
        }
    }
    for (int i = 0; i < n; i++) Wout[i] = W[i];
    for (int i = 0; i < n; i++) {
        double sd = W[i];
        double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

/* cvRodrigues2, 3x3 -> 3x1 (utils.py:242 `cv2.Rodrigues(par_r)`). */
void or_rodrigues_m2v(const double *Rin, double *rv) {
    double At[9], W[3], Vt[9], U[9], R[9];
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) At[i * 3 + j] = Rin[j * 3 + i];
    or_jacobi_svd(At, W, Vt, 3, 3);
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) U[i * 3 + j] = At[j * 3 + i];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += U[i * 3 + k] * Vt[k * 3 + j];
            R[i * 3 + j] = s;
        }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    if (s < 1e-5) {
        if (c > 0) { rx = ry = rz = 0; }
        else {
            double t;
            t = (R[0] + 1) * 0.5; rx = sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5; ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5; rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    rv[0] = rx; rv[1] = ry; rv[2] = rz;
}

/* cvRodrigues2, 3x1 -> 3x3 (inside cv2.projectPoints, utils.py:243). */
void or_rodrigues_v2m(const double *rv, double *R) {
    double rx = rv[0], ry = rv[1], rz = rv[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    /* glibc sincos(): what gcc emits for OpenCV's adjacent cos/sin calls at
     * -O2 (it differs from separate sin()/cos() in the last bit for some
     * arguments); called explicitly so every build agrees. */
    double c, s;
    sincos(theta, &s, &c);
    double c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int i = 0; i < 9; i++) {
        double e = (i % 4 == 0) ? 1.0 : 0.0;
        R[i] = (c * e + c1 * rrt[i]) + s * r_x[i];
    }
}

/* The rotation projectPoint actually projects with: R' = Rodrigues(Rodrigues(R)). */
void or_rodrigues_roundtrip(const double *R, double *Rp) {
    double rv[3];
    or_rodrigues_m2v(R, rv);
    or_rodrigues_v2m(rv, Rp);
}

/* cvProjectPoints2Internal with zero distortion (utils.py:241-244).
 * Rp = the Rodrigues round-tripped rotation; K's skew and third row are
 * ignored, as OpenCV does (fx=a[0], fy=a[4], cx=a[2], cy=a[5]). */
void or_project(const double *K, const double *Rp, const double *t, const double *M, double *out) {
    double X = M[0], Y = M[1], Z = M[2];
    double x = Rp[0] * X + Rp[1] * Y + Rp[2] * Z + t[0];
    double y = Rp[3] * X + Rp[4] * Y + Rp[5] * Z + t[1];
    double z = Rp[6] * X + Rp[7] * Y + Rp[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z; y *= z;
    out[0] = x * K[0] + K[2];
    out[1] = y * K[4] + K[5];
}

/* cvTriangulatePoints for one point (utils.py:238-239): 4x4 DLT, Jacobi SVD,
 * last right-singular vector (homogeneous, not normalised). */
void or_triangulate(const double *P1, const double *P2, const double *x1, const double *x2, double *X4) {
    double A[16];
    const double *P[2] = {P1, P2};
    const double *pt[2] = {x1, x2};
    for (int j = 0; j < 2; j++) {
        double x = pt[j][0], y = pt[j][1];
        for (int k = 0; k < 4; k++) {
            A[(j * 2 + 0) * 4 + k] = x * P[j][8 + k] - P[j][0 + k];
            A[(j * 2 + 1) * 4 + k] = y * P[j][8 + k] - P[j][4 + k];
        }
    }
    double At[16], W[4], Vt[16];
    for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) At[i * 4 + j] = A[j * 4 + i];
    or_jacobi_svd(At, W, Vt, 4, 4);
    for (int k = 0; k < 4; k++) X4[k] = Vt[3 * 4 + k];
}

/* ------------------------------------------------------------------------ */
/* numpy / reference restatements                                           */
/* ------------------------------------------------------------------------ */

static inline double dot3(const double *a, const double *b) {
    /* np.dot of two float64 3-vectors under OpenBLAS 0.3.29 (ddot kernel). */
    return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]));
}

/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src), n<=128 */
static double np_pairwise(const double *a, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
}

static double np_pairwise_any(const double *a, int n) {
    if (n <= 128) return np_pairwise(a, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_any(a, n2) + np_pairwise_any(a + n2, n - n2);
}

/* ctNcc (MVS2.py:39-43), bit-exact restatement of the numpy expression:
 *   d = (desc - np.mean(desc)) / np.std(desc); sum(d1*d2) / (n-1)
 * np.mean: exact integer sum / n.  np.std: sqrt(pairwise_sum((x-mean)^2)/n).
 * Python builtin sum(): sequential left-to-right. */
double or_ctncc(const uint8_t *a, const uint8_t *b, int n) {
    double xa[1024], xb[1024], sq[1024];
    int64_t sa = 0, sb = 0;
    for (int i = 0; i < n; i++) { sa += a[i]; sb += b[i]; }
    double ma = (double)sa / n, mb = (double)sb / n;
    for (int i = 0; i < n; i++) { xa[i] = (double)a[i] - ma; sq[i] = xa[i] * xa[i]; }
    double stda = sqrt(np_pairwise_any(sq, n) / n);
    for (int i = 0; i < n; i++) { xb[i] = (double)b[i] - mb; sq[i] = xb[i] * xb[i]; }
    double stdb = sqrt(np_pairwise_any(sq, n) / n);
    double s = 0;
    for (int i = 0; i < n; i++) s = s + (xa[i] / stda) * (xb[i] / stdb);
    return s / (n - 1);
}

/* Python int() of a float64 (truncation).  The reference raises on nan/inf;
 * such coordinates are reported as invalid here (documented deviation). */
static inline int py_int_ok(double v, long *out) {
    if (!(v > -1e15 && v < 1e15)) return 0;
    *out = (long)v;
    return 1;
}

/* getDescFeatures(gray, [[row, col]], wid) (HarrisFeatures.py:116-133):
 * bounds int(r)-w >= 0, int(r)+w+1 < H, int(c)-w > 0, int(c)+w+1 < W. */
int or_desc_window(int H, int W, double row, double col, int wid, long *r_out, long *q_out) {
    long r, q;
    if (!py_int_ok(row, &r) || !py_int_ok(col, &q)) return 0;
    if (!(r - wid >= 0 && r + wid + 1 < H && q - wid > 0 && q + wid + 1 < W)) return 0;
    *r_out = r; *q_out = q;
    return 1;
}

int or_get_desc(const uint8_t *gray_v, int H, int W, double row, double col, int wid, uint8_t *out) {
    long r, q;
    if (!or_desc_window(H, W, row, col, wid, &r, &q)) return 0;
    int k = 0;
    for (long y = r - wid; y <= r + wid; y++)
        for (long x = q - wid; x <= q + wid; x++) out[k++] = gray_v[y * W + x];
    return 1;
}

/* The scene: read-only arrays the photo test reads. */
typedef struct {
    int V, H, W;
    const uint8_t *gray;   /* V*H*W, view-major (the reference's per-view gray image) */
    const uint8_t *rgb;    /* V*H*W*3 (imgs, RGB) */
    const double *K;       /* V*9 */
    const double *Rp;      /* V*9, Rodrigues round-trip of Rraw */
    const double *Rraw;    /* V*9, par-file rotation */
    const double *t;       /* V*3 */
} or_scene;

/* MyPatch.photo_consistenecy_test (MVS2.py:62-77).  Every view is sampled at
 * the reference view's projection (the MVS2.py:68 quirk).  Writes the passing
 * view indices in increasing order; returns |V|. */
int or_photo_test(const or_scene *S, const double *c, int R, double thr, int wid,
                  int32_t *Vidx, double *xy, double *avg_out) {
    int n = (2 * wid + 1) * (2 * wid + 1);
    uint8_t base[1024], des[1024];
    double p[2];
    or_project(S->K + 9 * R, S->Rp + 9 * R, S->t + 3 * R, c, p);
    xy[0] = p[0]; xy[1] = p[1];
    int base_ok = or_get_desc(S->gray + (int64_t)R * S->H * S->W, S->H, S->W, p[1], p[0], wid, base);
    double avg = 0;
    int cnt = 0;
    for (int idx = 0; idx < S->V; idx++) {
        if (idx == R) continue;
        int ok = or_get_desc(S->gray + (int64_t)idx * S->H * S->W, S->H, S->W, p[1], p[0], wid, des);
        if (base_ok && ok) {
            double ncc = or_ctncc(base, des, n);
            if (ncc > thr) { avg += ncc; Vidx[cnt++] = idx; }
        }
    }
    if (cnt > 0) avg /= cnt;
    *avg_out = avg;
    return cnt;
}

/* Per-view ctNcc values of one candidate (nan where the reference computes
 * nan, -inf for idx == R or an invalid window): lets tests put a threshold
 * exactly on a reference value. */
void or_photo_ncc(const or_scene *S, const double *c, int R, int wid, double *ncc_out) {
    int n = (2 * wid + 1) * (2 * wid + 1);
    uint8_t base[1024], des[1024];
    double p[2];
    or_project(S->K + 9 * R, S->Rp + 9 * R, S->t + 3 * R, c, p);
    int base_ok = or_get_desc(S->gray + (int64_t)R * S->H * S->W, S->H, S->W, p[1], p[0], wid, base);
    for (int idx = 0; idx < S->V; idx++) {
        ncc_out[idx] = -INFINITY;
        if (idx == R || !base_ok) continue;
        if (or_get_desc(S->gray + (int64_t)idx * S->H * S->W, S->H, S->W, p[1], p[0], wid, des))
            ncc_out[idx] = or_ctncc(base, des, n);
    }
}

/* Batched photo test: the CPU baseline and the GPU parity checker.  mask has
 * ceil(V/64) words per candidate. */
void or_score_batch(const or_scene *S, int64_t n, const double *c, const int32_t *ref, double thr,
                    int wid, double *xy, uint64_t *mask, int32_t *count, double *avg, int nthreads) {
    int words = (S->V + 63) / 64;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64)
#endif
    for (int64_t i = 0; i < n; i++) {
        int32_t Vidx[OR_MAXV];
        int cnt = or_photo_test(S, c + 3 * i, ref[i], thr, wid, Vidx, xy + 2 * i, avg + i);
        for (int w = 0; w < words; w++) mask[i * words + w] = 0;
        for (int k = 0; k < cnt; k++) mask[i * words + Vidx[k] / 64] |= 1ull << (Vidx[k] % 64);
        count[i] = cnt;
    }
}

/* ------------------------------------------------------------------------ */
/* The MVS stage (MVS2.py:176-295): seeding + expansion + reconstruct        */
/* ------------------------------------------------------------------------ */

typedef struct {
    double c[3], n[3];
    int R;
    int nV;
    int32_t *V;      /* visible view indices (increasing) */
    double x, y;     /* projection into R, shared by every V entry (MVS2.py:68,74) */
    uint8_t color[3];
    double dist;
} or_patch;

typedef struct {
    /* patches, in creation order of the accepted objects */
    or_patch *p; int64_t np, cap;
    /* Q-table entries: (key, patch) in append order */
    int64_t *qkey; int64_t *qpatch; int64_t nq, qcap;
    /* stats */
    int64_t tests, pops, accepts;
} or_state;

static int64_t st_new_patch(or_state *st) {
    if (st->np == st->cap) {
        st->cap = st->cap ? st->cap * 2 : 4096;
        st->p = (or_patch *)realloc(st->p, st->cap * sizeof(or_patch));
    }
    return st->np++;
}

static void st_q_append(or_state *st, int64_t key, int64_t pid) {
    if (st->nq == st->qcap) {
        st->qcap = st->qcap ? st->qcap * 2 : 65536;
        st->qkey = (int64_t *)realloc(st->qkey, st->qcap * sizeof(int64_t));
        st->qpatch = (int64_t *)realloc(st->qpatch, st->qcap * sizeof(int64_t));
    }
    st->qkey[st->nq] = key; st->qpatch[st->nq] = pid; st->nq++;
}

typedef struct {
    int nci, ncj, cs;
    uint8_t *table;   /* V*nci*ncj, 1 = vacant (CellTable, MVS2.py:80-88) */
} or_cells;

static inline long py_floor_div(double v, int cs) { return (long)floor(v / cs); }

/* Python/numpy negative indexing: img[-1] is the last row (IndexError beyond). */
static inline long py_wrap(long i, long n) { return i < 0 ? i + n : i; }

/* CellTable.is_vacant (MVS2.py:90-96) */
static int cells_vacant(const or_cells *C, int v, long ci, long cj) {
    if (ci >= C->nci || ci < 0) return 0;
    if (cj >= C->ncj || cj < 0) return 0;
    return C->table[((int64_t)v * C->nci + ci) * C->ncj + cj];
}

/* CellTable.fill_with_point (MVS2.py:98-107).  The |V| appends under one key
 * of one call are collapsed to one (only first sight matters for
 * reconstruct_from_Q, MVS2.py:167). */
static int cells_fill(or_cells *C, or_state *st, int v, double col, double row, int64_t pid) {
    long ci = py_floor_div(col, C->cs), cj = py_floor_div(row, C->cs);
    if (ci >= C->nci || col < 0 || cj >= C->ncj || row < 0) return -1; /* reference: pdb trap */
    C->table[((int64_t)v * C->nci + ci) * C->ncj + cj] = 0;
    const or_patch *P = &st->p[pid];
    if (P->nV > 0) {
        long qi = py_floor_div(P->x, C->cs), qj = py_floor_div(P->y, C->cs);
        /* reconstruct_from_Q only visits in-table keys (MVS2.py:163-166) */
        if (qi >= 0 && qi < C->nci && qj >= 0 && qj < C->ncj)
            st_q_append(st, ((int64_t)v * C->nci + qi) * C->ncj + qj, pid);
    }
    return 0;
}

static void campos_of(const or_scene *S, int v, double *O) {
    /* -(par_r[i].T @ par_t[i]) (MVS2.py:189), OpenBLAS FMA-chain gemv */
    const double *R = S->Rraw + 9 * v, *t = S->t + 3 * v;
    for (int j = 0; j < 3; j++) O[j] = -fma(R[6 + j], t[2], fma(R[3 + j], t[1], R[j] * t[0]));
}

static int64_t run_photo(const or_scene *S, or_state *st, int64_t pid, double thr, int wid) {
    or_patch *P = &st->p[pid];
    int32_t Vidx[OR_MAXV];
    double xy[2], avg;
    int cnt = or_photo_test(S, P->c, P->R, thr, wid, Vidx, xy, &avg);
    P = &st->p[pid];
    P->nV = cnt;
    P->x = xy[0]; P->y = xy[1];
    P->V = NULL;
    if (cnt) {
        P->V = (int32_t *)malloc(cnt * sizeof(int32_t));
        memcpy(P->V, Vidx, cnt * sizeof(int32_t));
    }
    st->tests++;
    return cnt;
}

/* One expansion candidate (MVS2.py:329-369) for parent (pc, pn) whose V
 * entries carry pxy, hit view v, i = di: geometry, photo test (thr), accept
 * test.  Outputs X, nX, colour, projection, mask, count; returns accept. */
int or_expand_candidate(const or_scene *S, const double *pc, const double *pn, const double *pxy,
                        int v, int di, int cell_size, double scale, int wid, double thr,
                        double *X, double *nX, uint8_t *color, double *xy, uint64_t *mask,
                        int32_t *count) {
    const double *K = S->K + 9 * v, *R = S->Rraw + 9 * v, *t = S->t + 3 * v;
    double O[3];
    for (int j = 0; j < 3; j++) O[j] = -fma(R[6 + j], t[2], fma(R[3 + j], t[1], R[j] * t[0]));
    long ci = (long)floor(pxy[0] / cell_size), cj = (long)floor(pxy[1] / cell_size);
    double cc0 = cell_size * ((double)(ci + di) + 0.5);
    double cc1 = cell_size * ((double)(cj + di) + 0.5);
    double Cc[3], w[3], Pw[3], d[3];
    for (int q = 0; q < 3; q++) Cc[q] = fma(-R[6 + q], t[2], fma(-R[3 + q], t[1], (-R[q]) * t[0]));
    w[0] = cc0 - K[2]; w[1] = cc1 - K[5]; w[2] = (K[0] + K[4]) / 2;
    for (int q = 0; q < 3; q++) Pw[q] = fma(R[6 + q], w[2], fma(R[3 + q], w[1], R[q] * w[0])) + Cc[q];
    double nrm = sqrt((Pw[0] * Pw[0] + Pw[1] * Pw[1]) + Pw[2] * Pw[2]);
    for (int q = 0; q < 3; q++) d[q] = Pw[q] / nrm;
    double dot_out = dot3(d, pn);
    double cmo[3] = {pc[0] - O[0], pc[1] - O[1], pc[2] - O[2]};
    double tt = dot3(cmo, pn) / dot_out;
    for (int q = 0; q < 3; q++) X[q] = O[q] + tt * d[q];
    double e0 = X[0] - O[0], e1 = X[1] - O[1], e2 = X[2] - O[2];
    double dist = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
    for (int q = 0; q < 3; q++) nX[q] = (O[q] - X[q]) / dist;
    long cy = (long)cc1, cx = (long)cc0;
    cy = cy < 0 ? cy + S->H : cy; cx = cx < 0 ? cx + S->W : cx;
    const uint8_t *px = S->rgb + (((int64_t)v * S->H + cy) * S->W + cx) * 3;
    color[0] = px[0]; color[1] = px[1]; color[2] = px[2];
    int32_t Vidx[OR_MAXV];
    double avg;
    int cnt = or_photo_test(S, X, v, thr, wid, Vidx, xy, &avg);
    int words = (S->V + 63) / 64;
    for (int q = 0; q < words; q++) mask[q] = 0;
    for (int k = 0; k < cnt; k++) mask[Vidx[k] / 64] |= 1ull << (Vidx[k] % 64);
    *count = cnt;
    int vlb = S->V > 2 ? 3 : 2;
    double pm[3] = {pc[0] - X[0], pc[1] - X[1], pc[2] - X[2]};
    double nb = fabs(dot3(pm, pn) + dot3(pm, nX));
    double dd = sqrt((pm[0] * pm[0] + pm[1] * pm[1]) + pm[2] * pm[2]);
    return cnt >= vlb && nb < 0.1 && dd < 0.05 / scale;
}

typedef struct { double key[5]; int64_t pid; } heap_item;
static int cmp_heap(const void *a, const void *b) {
    const heap_item *x = (const heap_item *)a, *y = (const heap_item *)b;
    for (int k = 0; k < 5; k++) {
        if (x->key[k] < y->key[k]) return -1;
        if (x->key[k] > y->key[k]) return 1;
    }
    return 0;
}

/* Result of the stage. */
typedef struct {
    int64_t n_initial, n_all;
    double *initial;  /* n_initial*6 rows x,y,z,r,g,b */
    double *all;      /* n_all*6 */
    int64_t tests, pops, accepts, queue_left;
} or_result;

static int cmp_i64pair(const void *a, const void *b) {
    const int64_t *x = (const int64_t *)a, *y = (const int64_t *)b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    if (x[1] != y[1]) return x[1] < y[1] ? -1 : 1;
    return 0;
}

/* DensePointsWithMVS2 (MVS2.py:176-295) minus file IO.
 * tracks: track_off[n_tracks+1] into obs_view / obs_xy (the float32 values of
 * the SfM observations, widened to double as MVS2.py:229 does).
 * max_pops: min(cap, 100000) (MVS2.py:321). */
int or_mvs_stage(const or_scene *S, int64_t n_tracks, const int64_t *track_off, const int32_t *obs_view,
                 const double *obs_xy, int cell_size, double scale, int wid, int64_t max_pops,
                 or_result *res) {
    int V = S->V, H = S->H, W = S->W;
    or_state st; memset(&st, 0, sizeof st);
    or_cells C;
    C.cs = cell_size;
    C.nci = (int)ceil((double)(W - 1) / cell_size);   /* MVS2.py:88: ceil((col-1)/cs) */
    C.ncj = (int)ceil((double)(H - 1) / cell_size);
    C.table = (uint8_t *)malloc((size_t)V * C.nci * C.ncj);
    memset(C.table, 1, (size_t)V * C.nci * C.ncj);
    double *campos = (double *)malloc(sizeof(double) * 3 * V);
    for (int v = 0; v < V; v++) campos_of(S, v, campos + 3 * v);
    int vlb = V > 2 ? 3 : 2;   /* MVS2.py:200-203 */

    /* ---- seeding, MVS2.py:208-260 ---- */
    int64_t *initial = (int64_t *)malloc(sizeof(int64_t) * (n_tracks + 1));
    int64_t n_initial = 0;
    for (int64_t tr = 0; tr < n_tracks; tr++) {
        int64_t o0 = track_off[tr], o1 = track_off[tr + 1];
        if (o1 - o0 < 1) continue;
        int Rr = obs_view[o0];
        const double *base = obs_xy + 2 * o0;
        const double *O = campos + 3 * Rr;
        int nc = 0;
        heap_item *items = (heap_item *)malloc(sizeof(heap_item) * (o1 - o0));
        for (int64_t o = o0 + 1; o < o1; o++) {
            int k = obs_view[o];
            double P1[12], P2[12];
            /* getProjectionMatrix = K @ [r|t] (utils.py:234-236), OpenBLAS FMA chain */
            for (int rr = 0; rr < 3; rr++)
                for (int cc = 0; cc < 4; cc++) {
                    double e1[3], e2[3];
                    for (int q = 0; q < 3; q++) {
                        e1[q] = cc < 3 ? S->Rraw[9 * Rr + 3 * q + cc] : S->t[3 * Rr + q];
                        e2[q] = cc < 3 ? S->Rraw[9 * k + 3 * q + cc] : S->t[3 * k + q];
                    }
                    const double *K1 = S->K + 9 * Rr + 3 * rr, *K2 = S->K + 9 * k + 3 * rr;
                    P1[rr * 4 + cc] = fma(K1[2], e1[2], fma(K1[1], e1[1], K1[0] * e1[0]));
                    P2[rr * 4 + cc] = fma(K2[2], e2[2], fma(K2[1], e2[1], K2[0] * e2[0]));
                }
            double X4[4];
            or_triangulate(P1, P2, base, obs_xy + 2 * o, X4);
            int64_t pid = st_new_patch(&st);
            or_patch *P = &st.p[pid];
            memset(P, 0, sizeof *P);
            if (X4[3] == 0) { for (int q = 0; q < 3; q++) P->c[q] = 0 * X4[q]; }
            else { for (int q = 0; q < 3; q++) P->c[q] = X4[q] / X4[3]; }
            double d0 = P->c[0] - O[0], d1 = P->c[1] - O[1], d2 = P->c[2] - O[2];
            double dist = sqrt((d0 * d0 + d1 * d1) + d2 * d2);   /* utils.distance */
            for (int q = 0; q < 3; q++) P->n[q] = (O[q] - P->c[q]) / dist;
            P->R = Rr;
            P->dist = dist;
            long xi = (long)(float)obs_xy[2 * o], yi = (long)(float)obs_xy[2 * o + 1];  /* get_color: int(float32) */
            const uint8_t *px = S->rgb + (((int64_t)k * H + py_wrap(yi, H)) * W + py_wrap(xi, W)) * 3;
            P->color[0] = px[0]; P->color[1] = px[1]; P->color[2] = px[2];
            items[nc].key[0] = dist; items[nc].key[1] = P->c[0]; items[nc].key[2] = P->c[1];
            items[nc].key[3] = P->c[2]; items[nc].key[4] = Rr; items[nc].pid = pid;
            nc++;
        }
        qsort(items, nc, sizeof(heap_item), cmp_heap);   /* heap pops in key order */
        for (int q = 0; q < nc; q++) {
            int64_t pid = items[q].pid;
            int cnt = (int)run_photo(S, &st, pid, 0.4, wid);
            if (cnt >= vlb) {
                initial[n_initial++] = pid;
                or_patch *P = &st.p[pid];
                for (int h = 0; h < P->nV; h++) cells_fill(&C, &st, P->V[h], P->x, P->y, pid);
                break;
            }
        }
        free(items);
    }

    /* ---- patch_expansion, MVS2.py:308-404 ---- */
    int64_t qcap = 1 << 20, qhead = 0, qtail = 0;
    int64_t *queue = (int64_t *)malloc(sizeof(int64_t) * qcap);
    for (int64_t k = 0; k < n_initial; k++) queue[qtail++] = initial[k];
    int64_t iteration = 0;
    double dist_thr = 0.05 / scale;
    const int trace = getenv("MVS_TRACE") != NULL;
    while (qhead < qtail && iteration < max_pops) {
        iteration++;
        int64_t par = queue[qhead++];
        or_patch Pp = st.p[par];   /* copy: st.p may move */
        for (int h = 0; h < Pp.nV; h++) {
            int v = Pp.V[h];
            long ci = py_floor_div(Pp.x, cell_size), cj = py_floor_div(Pp.y, cell_size);
            for (int i = -1; i <= 1; i += 2) {
                for (int j = -1; j <= 1; j += 2) {
                    if (!cells_vacant(&C, v, ci + i, cj + j)) continue;
                    /* cell_center(ci+i, cj+i) -- the j->i quirk (MVS2.py:334) */
                    double cc0 = cell_size * ((double)(ci + i) + 0.5);
                    double cc1 = cell_size * ((double)(cj + i) + 0.5);
                    const double *K = S->K + 9 * v, *R = S->Rraw + 9 * v, *t = S->t + 3 * v;
                    double c_x = K[2], c_y = K[5], f_x = K[0], f_y = K[4];
                    double Cc[3], w[3], Pw[3], d[3];
                    for (int q = 0; q < 3; q++)   /* C = (-R^T @ t) (MVS2.py:351) */
                        Cc[q] = fma(-R[6 + q], t[2], fma(-R[3 + q], t[1], (-R[q]) * t[0]));
                    w[0] = cc0 - c_x; w[1] = cc1 - c_y; w[2] = (f_x + f_y) / 2;
                    for (int q = 0; q < 3; q++)   /* R^T @ w + C (MVS2.py:353) */
                        Pw[q] = fma(R[6 + q], w[2], fma(R[3 + q], w[1], R[q] * w[0])) + Cc[q];
                    double nrm = sqrt((Pw[0] * Pw[0] + Pw[1] * Pw[1]) + Pw[2] * Pw[2]);  /* vector_norm */
                    for (int q = 0; q < 3; q++) d[q] = Pw[q] / nrm;
                    const double *O = campos + 3 * v;
                    /* ray_plane_intersection (MVS2.py:302-306) */
                    double dot_out = dot3(d, Pp.n);
                    double cmo[3] = {Pp.c[0] - O[0], Pp.c[1] - O[1], Pp.c[2] - O[2]};
                    double tt = dot3(cmo, Pp.n) / dot_out;
                    double X[3];
                    for (int q = 0; q < 3; q++) X[q] = O[q] + tt * d[q];
                    int64_t pid = st_new_patch(&st);
                    or_patch *P = &st.p[pid];
                    memset(P, 0, sizeof *P);
                    memcpy(P->c, X, sizeof X);
                    double e0 = X[0] - O[0], e1 = X[1] - O[1], e2 = X[2] - O[2];
                    double dist = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
                    for (int q = 0; q < 3; q++) P->n[q] = (O[q] - X[q]) / dist;
                    P->R = v;
                    long cy = (long)cc1, cx = (long)cc0;   /* get_color: img[int(row)][int(col)] */
                    const uint8_t *px = S->rgb + (((int64_t)v * H + py_wrap(cy, H)) * W + py_wrap(cx, W)) * 3;
                    P->color[0] = px[0]; P->color[1] = px[1]; P->color[2] = px[2];
                    int cnt = (int)run_photo(S, &st, pid, 0.7, wid);
                    P = &st.p[pid];
                    /* accept test (MVS2.py:369) + is_patch_neighbor (MVS2.py:298-299) */
                    double pm[3] = {Pp.c[0] - P->c[0], Pp.c[1] - P->c[1], Pp.c[2] - P->c[2]};
                    double nb = fabs(dot3(pm, Pp.n) + dot3(pm, P->n));
                    double g0 = Pp.c[0] - P->c[0], g1 = Pp.c[1] - P->c[1], g2 = Pp.c[2] - P->c[2];
                    double dd = sqrt((g0 * g0 + g1 * g1) + g2 * g2);
                    if (trace) fprintf(stderr, "O pop %lld rec %lld v %d i %d j %d acc %d cnt %d cell %ld %ld\n",
                        (long long)iteration, (long long)par, v, i, j, (int)(cnt >= vlb && nb < 0.1 && dd < dist_thr), cnt,
                        (long)floor(P->x / cell_size), (long)floor(P->y / cell_size));
                    if (cnt >= vlb && nb < 0.1 && dd < dist_thr) {
                        st.accepts++;
                        for (int k = 0; k < P->nV; k++) {
                            cells_fill(&C, &st, P->V[k], P->x, P->y, pid);
                            if (qtail == qcap) {
                                qcap *= 2;
                                queue = (int64_t *)realloc(queue, sizeof(int64_t) * qcap);
                            }
                            queue[qtail++] = pid;
                        }
                        break;
                    } else {
                        /* rejected candidate objects are garbage in Python; drop it */
                        free(P->V);
                        st.np--;
                    }
                }
            }
        }
    }

    /* ---- reconstruct_from_Q, MVS2.py:159-173 ---- */
    int64_t *pairs = (int64_t *)malloc(sizeof(int64_t) * 2 * (st.nq + 1));
    for (int64_t k = 0; k < st.nq; k++) { pairs[2 * k] = st.qkey[k]; pairs[2 * k + 1] = k; }
    qsort(pairs, st.nq, 2 * sizeof(int64_t), cmp_i64pair);
    uint8_t *seen = (uint8_t *)calloc(st.np + 1, 1);
    res->all = (double *)malloc(sizeof(double) * 6 * (st.np + 1));
    int64_t na = 0;
    for (int64_t k = 0; k < st.nq; k++) {
        int64_t pid = st.qpatch[pairs[2 * k + 1]];
        if (seen[pid]) continue;
        seen[pid] = 1;
        const or_patch *P = &st.p[pid];
        double *row = res->all + 6 * na++;
        row[0] = P->c[0]; row[1] = P->c[1]; row[2] = P->c[2];
        row[3] = P->color[0]; row[4] = P->color[1]; row[5] = P->color[2];
    }
    res->n_all = na;
    res->initial = (double *)malloc(sizeof(double) * 6 * (n_initial + 1));
    for (int64_t k = 0; k < n_initial; k++) {
        const or_patch *P = &st.p[initial[k]];
        double *row = res->initial + 6 * k;
        row[0] = P->c[0]; row[1] = P->c[1]; row[2] = P->c[2];
        row[3] = P->color[0]; row[4] = P->color[1]; row[5] = P->color[2];
    }
    res->n_initial = n_initial;
    res->tests = st.tests; res->pops = iteration; res->accepts = st.accepts;
    res->queue_left = qtail - qhead;

    for (int64_t k = 0; k < st.np; k++) free(st.p[k].V);
    free(st.p); free(st.qkey); free(st.qpatch); free(pairs); free(seen);
    free(queue); free(initial); free(campos); free(C.table);
    return 0;
}

void or_result_free(or_result *r) {
    free(r->initial); free(r->all);
    r->initial = r->all = NULL;
}

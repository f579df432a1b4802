/* CPU restatement of the SfM front-end the MVS stage's seeds come from --
 * TEST INFRASTRUCTURE ONLY (the checker of the HIP path and the CPU baseline;
 * the product never links or calls this file).
 *
 *   or_harris_response   cv2.cornerHarris(gray_f32, 2, 3, 0.04)
 *                        (HarrisFeatures.py:139-141; OpenCV 4.x
 *                        imgproc/corner.cpp cornerEigenValsVecs + calcHarris,
 *                        scalar path)
 *   or_harris_points     getHarrisPoints (HarrisFeatures.py:135-161):
 *                        cv2.dilate(dst, None) (3x3, border ignored), keep
 *                        dst > float32(0.01) * dst.max() (NEP 50: the Python
 *                        float is cast to float32), np.where row-major order,
 *                        points [col, row]
 *   or_match_best        Match (HarrisFeatures.py:15-37) for one direction:
 *                        every pair's ctNcc in numpy's operation order
 *                        (or_ctncc, mvs_oracle.c), dist = ncc if ncc > thr,
 *                        best = argmax of the row
 *   or_sfm_pair          the body of StructureFromMotion's pair loop
 *                        (SFM.py:60-80) for one image pair: float32
 *                        triangulation (cv2.triangulatePoints on float32
 *                        points returns float32), w == 0 rows dropped,
 *                        point = X / w in float32, reprojection through
 *                        projectPoint (utils.py:241-244; projectPoints on a
 *                        float32 point returns float32) and the float32
 *                        np.linalg.norm of the residual against
 *                        MIN_REPROJECTION_ERROR
 *
 * Parity: pinned to the reference's own HarrisFeatures.py / SFM.py code run
 * in this container with the OpenCV stand-ins of tests/golden/standins/
 * (tests/golden/gen_sfm_golden.py); against a real OpenCV build it is
 * unpinned (OpenCV absent; the reference names no version).
 *
 * Ties in Match: numpy's argsort of equal keys is implementation-defined
 * (with AVX-512 x86-simd-sort it returns neither the first nor the last
 * index), so a row whose best value is shared, and a row with no ncc above
 * the threshold (an all-zero dist row), has no defined reference answer.
 * Here: ties -> smallest index, no pass -> -1 (no match); such rows are
 * reported through `flags` and excluded from the golden comparison.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

double or_ctncc(const uint8_t *a, const uint8_t *b, int n);   /* mvs_oracle.c */
void or_triangulate(const double *P1, const double *P2, const double *x1, const double *x2, double *X4);
void or_rodrigues_roundtrip(const double *R, double *Rp);
void or_project(const double *K, const double *Rp, const double *t, const double *M, double *out);

static inline int refl101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
}

void or_harris_response(const uint8_t *gray, int H, int W, double k, float *resp) {
    float *dx = malloc(sizeof(float) * (size_t)H * W), *dy = malloc(sizeof(float) * (size_t)H * W);
    float *cv = malloc(sizeof(float) * 3 * (size_t)H * W);
    /* Sobel 3x3 with scale 1/8 folded into the smoothing taps: exact in float32
     * (integer gray, power-of-two scale) */
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float gx = 0.f, gy = 0.f;
            for (int u = -1; u <= 1; u++) {
                const int yy = refl101(y + u, H);
                const float sm = u == 0 ? 0.25f : 0.125f;
                const float d = (float)gray[(size_t)yy * W + refl101(x + 1, W)] -
                                (float)gray[(size_t)yy * W + refl101(x - 1, W)];
                gx += sm * d;
            }
            for (int u = -1; u <= 1; u++) {
                const int xx = refl101(x + u, W);
                const float sm = u == 0 ? 0.25f : 0.125f;
                const float d = (float)gray[(size_t)refl101(y + 1, H) * W + xx] -
                                (float)gray[(size_t)refl101(y - 1, H) * W + xx];
                gy += sm * d;
            }
            dx[(size_t)y * W + x] = gx;
            dy[(size_t)y * W + x] = gy;
        }
    for (size_t p = 0; p < (size_t)H * W; p++) {
        cv[3 * p] = dx[p] * dx[p];
        cv[3 * p + 1] = dx[p] * dy[p];
        cv[3 * p + 2] = dy[p] * dy[p];
    }
    /* boxFilter 2x2, unnormalised, anchor (1,1): rows y-1..y, cols x-1..x;
     * every partial sum is exact in float32 */
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float s[3] = {0.f, 0.f, 0.f};
            for (int u = -1; u <= 0; u++)
                for (int v = -1; v <= 0; v++) {
                    const size_t q = (size_t)refl101(y + u, H) * W + refl101(x + v, W);
                    for (int c = 0; c < 3; c++) s[c] += cv[3 * q + c];
                }
            const float a = s[0], b = s[1], c = s[2];
            const float acbb = a * c - b * b;
            const double t = (double)(a + c);
            resp[(size_t)y * W + x] = (float)((double)acbb - k * t * t);
        }
    free(dx);
    free(dy);
    free(cv);
}

/* returns the number of points; writes min(n, cap) [col, row] pairs */
int64_t or_harris_points(const uint8_t *gray, int H, int W, int32_t *out, int64_t cap) {
    float *r = malloc(sizeof(float) * (size_t)H * W), *d = malloc(sizeof(float) * (size_t)H * W);
    or_harris_response(gray, H, W, 0.04, r);
    float mx = -INFINITY;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float m = -INFINITY;
            for (int u = -1; u <= 1; u++)
                for (int v = -1; v <= 1; v++) {
                    const int yy = y + u, xx = x + v;
                    if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
                    const float z = r[(size_t)yy * W + xx];
                    if (z > m) m = z;
                }
            d[(size_t)y * W + x] = m;
            if (m > mx) mx = m;
        }
    const float thr = 0.01f * mx;
    int64_t n = 0;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            if (d[(size_t)y * W + x] > thr) {
                if (n < cap) {
                    out[2 * n] = x;
                    out[2 * n + 1] = y;
                }
                n++;
            }
    free(r);
    free(d);
    return n;
}

/* Match(desc1, desc2, thr) one direction: best[i] = argmax_j dist[i, j]
 * (ties -> smallest j), -1 if no ncc > thr.  flags[i]: 1 = tie at the
 * maximum, 2 = no pass (the reference's answer is implementation-defined). */
void or_match_best(const uint8_t *d1, int64_t n1, const uint8_t *d2, int64_t n2, int npx,
                   double thr, int32_t *best, double *best_ncc, uint8_t *flags) {
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t i = 0; i < n1; i++) {
        double bv = 0.0;
        int64_t bj = -1;
        int tie = 0;
        for (int64_t j = 0; j < n2; j++) {
            const double v = or_ctncc(d1 + i * npx, d2 + j * npx, npx);
            if (!(v > thr)) continue;
            if (bj < 0 || v > bv) {
                bv = v;
                bj = j;
                tie = 0;
            } else if (v == bv) {
                tie = 1;
            }
        }
        best[i] = (int32_t)bj;
        if (best_ncc) best_ncc[i] = bj < 0 ? 0.0 : bv;
        if (flags) flags[i] = (uint8_t)(bj < 0 ? 2 : tie ? 1 : 0);
    }
}

/* SFM.py:60-80 for one pair: P1 = K_A [R_A | t_A], P2 = K_B [R_B | t_B]
 * (getProjectionMatrix), q / tr float32 [x, y] correspondences.
 * keep[i] = 1 if the point is added (w != 0 and both reprojection errors
 * <= max_err); pt[i] = float32 point. */
void or_sfm_pair(const double *KA, const double *RA, const double *tA, const double *KB,
                 const double *RB, const double *tB, int64_t n, const float *q, const float *tr,
                 double max_err, float *pt, uint8_t *keep) {
    double P1[12], P2[12], RpA[9], RpB[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) {
            /* getProjectionMatrix = K @ [R | t] (utils.py:234-236) as OpenBLAS
             * evaluates it: an FMA chain per entry (as in or_mvs_stage) */
            double e1[3], e2[3];
            for (int k = 0; k < 3; k++) {
                e1[k] = c < 3 ? RA[3 * k + c] : tA[k];
                e2[k] = c < 3 ? RB[3 * k + c] : tB[k];
            }
            const double *K1 = KA + 3 * r, *K2 = KB + 3 * r;
            P1[4 * r + c] = fma(K1[2], e1[2], fma(K1[1], e1[1], K1[0] * e1[0]));
            P2[4 * r + c] = fma(K2[2], e2[2], fma(K2[1], e2[1], K2[0] * e2[0]));
        }
    or_rodrigues_roundtrip(RA, RpA);
    or_rodrigues_roundtrip(RB, RpB);
    for (int64_t i = 0; i < n; i++) {
        const double x1[2] = {q[2 * i], q[2 * i + 1]}, x2[2] = {tr[2 * i], tr[2 * i + 1]};
        double X4[4];
        or_triangulate(P1, P2, x1, x2, X4);
        const float w = (float)X4[3];
        keep[i] = 0;
        pt[3 * i] = pt[3 * i + 1] = pt[3 * i + 2] = 0.f;
        if (w == 0.f) continue;
        float p[3];
        for (int k = 0; k < 3; k++) p[k] = (float)X4[k] / w;
        for (int k = 0; k < 3; k++) pt[3 * i + k] = p[k];
        const double M[3] = {p[0], p[1], p[2]};
        double oa[2], ob[2];
        or_project(KA, RpA, tA, M, oa);
        or_project(KB, RpB, tB, M, ob);
        const float ea0 = (float)oa[0] - q[2 * i], ea1 = (float)oa[1] - q[2 * i + 1];
        const float eb0 = (float)ob[0] - tr[2 * i], eb1 = (float)ob[1] - tr[2 * i + 1];
        const float na = sqrtf(ea0 * ea0 + ea1 * ea1), nb = sqrtf(eb0 * eb0 + eb1 * eb1);
        keep[i] = ((double)na > max_err || (double)nb > max_err) ? 0 : 1;
    }
}

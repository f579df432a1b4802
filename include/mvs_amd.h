/*
 * mvs_amd.h -- C-ABI of the MI355X-native MVS patch-expansion library
 * (libmvs_amd.so, built from
 *  simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/csrc).
 *
 * The reference (MarvinChung/simple-implementation-of-structure-from-motion-
 * and-multi-view-stereo-by-python) is pure Python with no FFI; each entry point
 * below names the Python interface it replaces.  Conventions:
 *   - plain pointers and sizes, no torch / C++ types;
 *   - every call returns 0 on success or a negative status
 *     (MVS_E_ARG, MVS_E_HIP, MVS_E_UNSUPPORTED, MVS_E_NOMEM); the message is in
 *     mvs_last_error(ctx) (or mvs_last_error(NULL) when create failed);
 *   - no C++ exception crosses the ABI;
 *   - one context per device, driven by one host thread; *_device calls are
 *     ordered on the caller's HIP stream (NULL = the context's stream).
 *
 * Arrays follow the reference's numpy conventions: K/R row-major 3x3 per view
 * (V*9 doubles), t 3 per view, images V*H*W*3 uint8 RGB (main.py:17-18), view
 * index = position in the sorted image list = par-file row - 1 (utils.py:72-80).
 */
#ifndef MVS_AMD_H
#define MVS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVS_OK 0
#define MVS_E_ARG (-1)
#define MVS_E_HIP (-2)
#define MVS_E_UNSUPPORTED (-3)
#define MVS_E_NOMEM (-4)
#define MVS_E_DIVZERO (-5)   /* the reference would raise ZeroDivisionError (filter_out_outlier) */

typedef struct mvs_ctx mvs_ctx;
typedef struct mvs_stage_result mvs_stage_result;
typedef struct mvs_stage mvs_stage;

/* Library version string. */
const char* mvs_version(void);

/* Scene setup: replaces the per-call work the reference redoes on every photo
 * test -- read_pars (utils.py:56-81, called at MVS2.py:178/309), the per-call
 * full-frame copy + cvtColor(BGR2GRAY) (HarrisFeatures.py:124-125) and
 * cv2.Rodrigues(par_r) (utils.py:242).  Uploads the images once, builds the
 * device gray stack (OpenCV BGR2GRAY fixed-point formula applied to the RGB
 * data, as the reference does) and the per-view camera table.
 * Rp may be NULL (the library computes R' = Rodrigues(Rodrigues(R))).
 * 1 <= V <= 256, 16 <= H, W <= 65536. */
int mvs_ctx_create(int device, int V, int H, int W, const uint8_t* rgb, const double* K,
                   const double* R, const double* t, const double* Rp, mvs_ctx** out);
void mvs_ctx_destroy(mvs_ctx* ctx);
const char* mvs_last_error(const mvs_ctx* ctx);
/* Copies the rotations the projection uses (V*9) -- for parity tests. */
int mvs_ctx_rproj(const mvs_ctx* ctx, double* Rp);
/* The device part of the scene setup again, from the resident RGB images:
 * the gray stack and its signed view-major copy (k_build_scene).  For
 * measuring a cold sweep (setup + scoring); stream-ordered (NULL = the
 * context's stream). */
int mvs_ctx_rebuild(mvs_ctx* ctx, void* stream);

/* Batched MyPatch.photo_consistenecy_test (MVS2.py:62-77): for candidate i
 * with centre c[3i..3i+2] and reference view ref[i], project into ref[i]
 * (projectPoint, utils.py:241-244), take the (2*wid+1)^2 windows of every view
 * at that pixel (getDescFeatures, HarrisFeatures.py:116-133; all views at the
 * reference view's pixel, MVS2.py:68), and keep the views idx != ref with
 * ctNcc > min_ncc (MVS2.py:39-43, 72).
 * Outputs: xy[2i..] = projection (the x, y of every V entry, MVS2.py:74);
 * mask[i*words + w] bit b = view 64w+b passed (words = ceil(V/64));
 * count[i] = |V|; avg[i] = mean ncc of the passing views (avg_ncc_score).
 * Host pointers; synchronous. wid in 1..5. */
int mvs_score(mvs_ctx* ctx, int64_t n, const double* c, const int32_t* ref, int wid,
              double min_ncc, double* xy, uint64_t* mask, int32_t* count, double* avg);
/* Same on device pointers (e.g. torch tensor data_ptr()), stream-ordered.
 * Calls on different streams are ordered too: a call waits for the previous
 * call's use of the context's scratch (an event on that call's stream).
 * d_avg may be NULL when avg_ncc_score is not needed (it only feeds the
 * disabled filter_out_outlier, MVS2.py:281).
 * Device memory: the first tiled call with a given wid builds that wid's
 * window-moment tables, kept for the context's life: (H*W + 16) * VP
 * entries (VP = V rounded up to 16, or to 64 at V > 64) of 10 B at
 * V <= 64 (S_b int16 + w binary64) or 6 B at V > 64 (S_b int16 + D int32)
 * -- 147 MB per wid for dinoRing (48 x 640 x 480), 3.2 GB for
 * 256 x 1920 x 1080.  Past 2^31
 * entries, or when the allocation fails, that scene is scored with the
 * in-kernel moments instead (same results, slower). */
int mvs_score_device(mvs_ctx* ctx, int64_t n, const double* d_c, const int32_t* d_ref, int wid,
                     double min_ncc, double* d_xy, uint64_t* d_mask, int32_t* d_count,
                     double* d_avg, void* stream);
/* The same photo test with one record per candidate instead of three arrays:
 * d_rec[i * (words + 1) ...] = [mask words of i, avg_ncc_score as binary64
 * bits]; |V| = the popcount of the mask words.  One 16-B store per candidate
 * at V <= 64 (the scorer's output stores are scattered by candidate id).
 * d_rec 16-B aligned; mvs_pack_accepted reads it with d_count = NULL. */
int mvs_score_device_rec(mvs_ctx* ctx, int64_t n, const double* d_c, const int32_t* d_ref, int wid,
                         double min_ncc, double* d_xy, int64_t* d_rec, void* stream);
/* CellTable.filter_out_outlier (MVS2.py:132-158) on the host, over n accepted
 * patches in fill order (what the stage's opt-in filter mode runs between
 * the expansion and reconstruct_from_Q): patch e has cell[2e..2e+1] =
 * which_cell of its projection (MVS2.py:113), mask[e*words..] its V list,
 * count[e] = |V|, avg[e] = avg_ncc_score, c[3e..], nrm[3e..].  Out:
 * alive[e] = 0 for the removed patches, stats[0] = removed patches,
 * stats[1] = "remove a outlier" lines the reference prints.  The
 * reference's ZeroDivisionError (a filled cell emptied before its visit,
 * MVS2.py:144) is MVS_E_DIVZERO.  Host pointers; no GPU needed. */
int mvs_filter_outliers(int64_t n, int words, int nci, int ncj, const int32_t* cell,
                        const uint64_t* mask, const int32_t* count, const double* avg,
                        const double* c, const double* nrm, uint8_t* alive, int64_t* stats);
/* The multi-GPU sweep's exchange record set (no reference counterpart: the
 * reference is single-process).  The accepted candidates
 * (count >= vlb, MVS2.py:256/369) of a slice of n scored candidates are
 * packed into d_out[(cap + 1) * width] int64 with width = 1 + words +
 * (d_c ? 3 : 0): row 0 = [accepted, n, 0...], rows 1.. = [offset + i, mask
 * words of i, and with d_c (the slice's n*3 centres, the candidates' 3D
 * points) the binary64 bits of x, y, z] (40 B at V <= 64; d_c = NULL: 16 B,
 * the receiver regenerating a point from its global index).  Row order: each
 * chunk of 8,192 candidates in index order, the chunks in the order they
 * reserve their rows (one atomic each; nothing waits for another chunk), so
 * the set is exact and the order is not: a receiver that needs index order
 * sorts by the first column (parallel.PointsExchange.result does).
 * d_count = NULL: d_mask is mvs_score_device_rec's records (words + 1 int64
 * each) and |V| their popcount.
 * Device pointers, stream-ordered, no host synchronisation (the accepted
 * total is in the header; a slice with more than cap accepted keeps cap of
 * them).  Calls on one context are ordered across streams (their counter is
 * the context's).  Feeds the all-gather of parallel.PointsExchange. */
int mvs_pack_accepted(mvs_ctx* ctx, int64_t n, int64_t offset, const int32_t* d_count,
                      const uint64_t* d_mask, const double* d_c, int vlb, int64_t cap, int64_t* d_out,
                      void* stream);
/* Measurement only (bench.py exchange.overlap_proxy): copies bytes (a
 * multiple of 16) from d_src to d_dst with a kernel of `workgroups`
 * 256-thread workgroups on `stream` -- the CU footprint of a collective's
 * kernel, run beside the scoring kernels on one GPU. */
int mvs_proxy_copy(void* d_dst, const void* d_src, int64_t bytes, int workgroups, void* stream);
/* The persistent tiled scorers' grid: `workgroups` > 0 holds them to that
 * many workgroups (at two per CU, the CUs of a CU-masked scoring stream), 0
 * restores the default (every CU, twice).  Multi-GPU steps score on a stream
 * whose CU mask leaves a few CUs to the exchange's pack and RCCL's kernels
 * (parallel.cu_masked_stream); no reference counterpart. */
int mvs_set_scorer_grid(mvs_ctx* ctx, int workgroups);
/* Kernel timing (measurement only): while enabled, every enable-th scoring
 * call (enable = 1: every call) records a HIP event pair on its stream
 * immediately around the dominant scoring kernel (k_score_mma / k_score_mma_v
 * for batches of >= 2048 candidates, else k_score); sampling keeps the
 * events' own stream time out of most calls of a timed loop.  enable > 0
 * resets the record and turns it on; 0 turns it off (the record stays
 * readable).  mvs_kernel_time synchronises the recorded events and returns
 * the summed kernel time and the number of timed launches; mvs_timed_kernel
 * names the kernel the last recorded pair bracketed. */
int mvs_kernel_timing(mvs_ctx* ctx, int enable);
int mvs_kernel_time(mvs_ctx* ctx, double* total_ms, int64_t* launches);
const char* mvs_timed_kernel(const mvs_ctx* ctx);
/* Number of per-view NCC decisions that fell inside the direct scorer's guard
 * band around the threshold (relative 1e-11 on the squared comparison; 1e-9
 * absolute when min_ncc < 0.01) and were re-evaluated in numpy order since the
 * context was created.  (The tiled scorer's own band, 2e-6 relative on its
 * binary32 comparison, sends a candidate to the direct scorer.) */
int64_t mvs_exact_hits(mvs_ctx* ctx);
/* A caller stream that a *_device call has used is about to be destroyed
 * (hipStreamDestroy): the context waits for that stream's work on its
 * scratch and pack areas now.  The context orders calls made on different
 * streams by an event recorded lazily on the stream that used an area last,
 * when the next call comes from another stream; a destroyed stream cannot
 * take that record (its handle may even be reused by a new stream), so a
 * caller that retires streams calls this first, on every context the stream
 * has used (parallel.MaskedStream.close does).  Streams the caller keeps
 * need nothing. */
int mvs_stream_retiring(mvs_ctx* ctx, void* stream);

/* Direct-path statistics of the tiled scorers since the context was created
 * (device work ordered before this call on the context's stream is counted;
 * call after synchronising the streams that scored): out[0] = candidates
 * re-scored by the direct path (k_score_fix: the tiled scorer's guard band
 * plus bucket overflow), out[1] = of them bucket overflow, out[2] = tiled
 * batches.  Diagnostic (bench.py reports the guard-band rate per sweep). */
int mvs_scorer_stats(mvs_ctx* ctx, int64_t* out);

/* ctNcc (MVS2.py:39-43) on n explicit window pairs of npx (<= 128) uint8
 * pixels each (device pointers).  ncc[i] = closed-form value (numpy-order
 * value if force_exact or within 1e-9 of thr; nan for a constant window);
 * pass[i] = ncc > thr. */
int mvs_ncc_windows(int64_t n, int npx, const uint8_t* d_a, const uint8_t* d_b, double thr,
                    int force_exact, double* d_ncc, uint8_t* d_pass, void* stream);

/* DensePointsWithMVS2 (MVS2.py:176-295) without file IO: seeding from the SfM
 * tracks (MVS2.py:205-260), patch_expansion (MVS2.py:308-404, FIFO capped at
 * min(max_pops, 100000) pops) and reconstruct_from_Q ordering
 * (MVS2.py:159-173).  Tracks: track t owns observations
 * [track_off[t], track_off[t+1]); obs_view = image index, obs_xy = (x, y)
 * float32 pairs (GlobalSet point2d_list); element 0 is the reference view.
 * cell_size / scale / wid as args.cell_size, args.scale and the photo test's
 * window half-width (5 in the reference). */
int mvs_stage_run(mvs_ctx* ctx, int64_t n_tracks, const int64_t* track_off,
                  const int32_t* obs_view, const float* obs_xy, int cell_size, double scale,
                  int wid, int64_t max_pops, mvs_stage_result** out);
/* which = 0: initial_patches rows, 1: all_patches rows (x,y,z,r,g,b float64).
 * The rows are ordered and gathered on the device; mvs_stage_rows copies them
 * into a host buffer, mvs_stage_rows_device into a device buffer
 * (stream-ordered). */
int64_t mvs_stage_count(const mvs_stage_result* res, int which);
int mvs_stage_rows(const mvs_stage_result* res, int which, double* rows);
int mvs_stage_rows_device(const mvs_stage_result* res, int which, double* d_rows, void* stream);
/* stats[0..7] = pops, reference-equivalent photo tests, accepted patches,
 * queue entries left, candidates scored on the GPU, sweeps, seed candidates,
 * exact-path decisions. */
int mvs_stage_stats(const mvs_stage_result* res, int64_t* stats);
/* Host wall seconds per stage phase: times[0] seeding, [1] ordered commit and
 * sweep planning, [2] GPU sweeps, [3] sweep copy-back, [4] output ordering,
 * [5] the whole call. */
int mvs_stage_times(const mvs_stage_result* res, double* times);
void mvs_stage_free(mvs_stage_result* res);

/* Stage options of a context, for the stage runs that follow (mvs_stage_run,
 * mvs_stage_begin ... mvs_stage_finish).  MVS_STAGE_FILTER_OUTLIERS runs
 * CellTable.filter_out_outlier (MVS2.py:132-158) between the expansion and the
 * reconstruction, as if the reference's commented-out call at MVS2.py:281
 * were enabled (avg_ncc_score then follows the reference's arithmetic
 * exactly).  A filled cell whose patches were all removed before it is
 * visited makes the reference raise ZeroDivisionError: MVS_E_DIVZERO. */
#define MVS_STAGE_FILTER_OUTLIERS 1
/* avg_ncc_score (MVS2.py:62-76) in the reference's own arithmetic for n scored
 * candidates (host arrays: ref, xy (n*2) and mask (n*words) as mvs_score
 * returned them): ctNcc in numpy's order for every view of the mask, summed
 * in view order from 0, divided by the view count (0 for an empty mask).
 * mvs_score's avg agrees with it to 1e-12; this one is bit-exact. */
int mvs_exact_avg(mvs_ctx* ctx, int64_t n, const int32_t* ref, const double* xy, const uint64_t* mask,
                  int wid, double* avg);
int mvs_stage_set_options(mvs_ctx* ctx, int flags);
/* out[0] = outlier patches removed, out[1] = "remove a outlier" lines the
 * reference prints for them (|V|^2 each). */
int mvs_stage_filter_stats(const mvs_stage_result* res, int64_t* out);

/* The same stage in steps, for several GPUs (one process and one context per
 * GPU).  Every rank calls mvs_stage_begin with the same inputs
 * and its (rank, world), then loops:
 *   nj = mvs_stage_plan(st)          commit in reference order until the FIFO
 *                                    head needs unscored children; plan the next
 *                                    sweep of nj child jobs (0: stage finished)
 *   mvs_stage_score_slice(st, out)   the geometry of every child of the sweep
 *                                    (it depends only on parent records, which
 *                                    every rank holds) and the photo + accept
 *                                    test of this rank's contiguous slice
 *                                    (rank r: jobs [r*b + min(r, x),
 *                                    ... + b + (r < x)), b = nj / world,
 *                                    x = nj % world); the slice's photo-test
 *                                    masks go to the device buffer
 *                                    out[ceil(nj/world)][width] (world > 1;
 *                                    may be NULL when world == 1)
 *   <all-gather the slices, e.g. RCCL>
 *   mvs_stage_ingest(st, all)        all[world][ceil(nj/world)][width] (device):
 *                                    the other ranks' masks into the record
 *                                    table, their counts (popcount) and accept
 *                                    tests; `all` must be complete when called
 *                                    (the context's stream waits for no other
 *                                    stream)
 * and ends with mvs_stage_finish (same result as mvs_stage_run) and
 * mvs_stage_destroy.  width = mvs_stage_record_width(st) int64 words (the
 * mask words: 8 B per child at V <= 64).  Seeding
 * is replicated on every rank; the commit is identical on every rank because
 * it reads identical records.  Calls are synchronous. */
int mvs_stage_begin(mvs_ctx* ctx, int64_t n_tracks, const int64_t* track_off,
                    const int32_t* obs_view, const float* obs_xy, int cell_size, double scale,
                    int wid, int64_t max_pops, int rank, int world, mvs_stage** out);
int64_t mvs_stage_plan(mvs_stage* st);
int mvs_stage_record_width(const mvs_stage* st);
int mvs_stage_score_slice(mvs_stage* st, int64_t* d_out);
int mvs_stage_ingest(mvs_stage* st, const int64_t* d_all);
int mvs_stage_finish(mvs_stage* st, mvs_stage_result** out);
void mvs_stage_destroy(mvs_stage* st);

/* patch_expansion candidates (MVS2.py:329-369) for explicit jobs: job k =
 * (parent job_parent[k], hit view job_view[k], i = job_di[k] in {-1,+1}).
 * Parents: centre pc, normal pn, pxy = projection into the parent's
 * reference view (the x, y of its V entries).  Per job: X, nX (n of the new
 * patch), colour (img[int(cc1)][int(cc0)]), projection xy, mask/count of the
 * photo test at min_ncc, accept = |V| >= vlb && is_patch_neighbor(0.1) &&
 * |pc - X| < 0.05/scale.  Host pointers; wid 3 or 5. */
int mvs_expand_candidates(mvs_ctx* ctx, int64_t n_parents, const double* pc, const double* pn,
                          const double* pxy, int64_t n_jobs, const int32_t* job_parent,
                          const int32_t* job_view, const int32_t* job_di, int cell_size,
                          double scale, int wid, double min_ncc, double* X, double* nX,
                          uint8_t* color, double* xy, uint64_t* mask, int32_t* count,
                          uint8_t* accept);

/* Host geometry the stage uses, exported for parity tests:
 * cv2.Rodrigues round trip (utils.py:242-243) and cv2.triangulatePoints for one
 * point (utils.py:238-239, homogeneous 4-vector). */
int mvs_rodrigues_roundtrip(const double* R, double* Rp);
int mvs_triangulate(const double* P1, const double* P2, const double* x1, const double* x2,
                    double* X4);

/* ---- SfM front-end: the producer of the stage's seed tracks ----
 * (BASELINE config 5: HarrisFeatures + SFM.py feeding MVS; the reference's
 * default SfM matcher is OpenCV ORB/FLANN/RANSAC, SFM.py:56, utils.py:160-232)
 *
 * getHarrisPoints(imgs[view]) (HarrisFeatures.py:135-161) on the GPU:
 * cv2.cornerHarris(gray, 2, 3, 0.04), 3x3 dilate, keep > float32(0.01) * max,
 * np.where row-major order.  out: [col, row] int32 pairs (host), at most cap
 * of them; *n_out = the total (call with cap 0 to size the buffer). */
int mvs_harris_points(mvs_ctx* ctx, int view, int32_t* out, int64_t cap, int64_t* n_out);

/* MatchTwoSided(getDescFeatures(imgs[view_a], pts_a, wid),
 *               getDescFeatures(imgs[view_b], pts_b, wid), thr)
 * (HarrisFeatures.py:15-67) on the GPU.  pts_* are [row, col] int32 (host),
 * all inside getDescFeatures' bounds (else MVS_E_ARG).  m12[i] = j when j is
 * i's best match and i is j's, else -1; best12 / best21 (may be NULL): the
 * one-sided argmax of ncc > thr (ties -> smallest index, -1 when no ncc
 * exceeds thr; numpy's argsort leaves both cases implementation-defined). */
int mvs_match_two_sided(mvs_ctx* ctx, int view_a, const int32_t* pts_a, int64_t n_a, int view_b,
                        const int32_t* pts_b, int64_t n_b, int wid, double thr, int32_t* m12,
                        int32_t* best12, int32_t* best21);

/* One image pair of StructureFromMotion's loop (SFM.py:60-80), host:
 * P = K [R | t] per view (getProjectionMatrix), cv2.triangulatePoints of
 * the float32 correspondences q (view A) / tr (view B) (float32 result),
 * point = X / w; keep[i] = 1 when w != 0 and both projectPoint residuals
 * (float32 norm) are <= max_err (MIN_REPROJECTION_ERROR).  pt: float32 (n, 3).
 * K, R row-major 3x3, t 3 doubles. */
int mvs_sfm_pair(const double* KA, const double* RA, const double* tA, const double* KB,
                 const double* RB, const double* tB, int64_t n, const float* q, const float* tr,
                 double max_err, float* pt, uint8_t* keep);

#ifdef __cplusplus
}
#endif
#endif /* MVS_AMD_H */

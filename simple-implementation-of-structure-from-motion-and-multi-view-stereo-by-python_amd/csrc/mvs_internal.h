// Internal declarations shared by the HIP kernels (mvs_kernels.hip,
// sfm_kernels.hip) and the host engine (mvs_engine.cpp).  Not part of the
// public C-ABI (include/mvs_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MVS_MAX_VIEWS 256
#define MVS_MAX_WID 5

// Per-view camera constants, laid out for wave-uniform (scalar) loads.
// All values are computed on the host in the reference's operation order
// (see mvs_engine.cpp: build_cameras).
struct CamDev {
    double Rp[9];   // Rodrigues round-trip of R (what cv2.projectPoints uses, utils.py:242-243)
    double t[3];
    double fx, fy, cx, cy;   // OpenCV projectPoints reads a[0], a[4], a[2], a[5]
    double R[9];    // par-file rotation (MVS2.py:351-353)
    double O[3];    // camera_pos = -(R^T t)      (MVS2.py:189)
    double C[3];    // (-R^T) @ t                 (MVS2.py:351)
    double fbar;    // (f_x + f_y)/2              (MVS2.py:353)
    double pad[3];
};

// Device-resident scene, two layouts of the same gray images (OpenCV's
// BGR2GRAY fixed-point formula on the RGB data, HarrisFeatures.py:125):
//  * stack[y][k][v][4] = gray_v(y, 4k..4k+3): one window row of every view is
//    one contiguous run (the direct per-candidate scorers, lane = view);
//  * gv[v][y][x] = g - 128 as a signed byte (the i8 operands of the tiled
//    matrix-core scorer), row pitch Wp (a multiple of 16) with 8 pad bytes
//    left of column 0 and >= 24 right of column W-1: a tile region row of
//    one view (columns x0-8 .. x0+23, x0 a multiple of 16) is two aligned
//    16-byte pieces.  gv points at column 0.
struct SceneDev {
    int V, H, W;
    int Wq;            // quads per row, incl. one zero pad quad
    int64_t row_bytes; // Wq * V * 4
    const uint8_t* stack;
    const uint8_t* rgb;      // V*H*W*3 (colour lookups of expansion candidates)
    const CamDev* cams;
    const uint8_t* gv;
    int Wp;
};

// Inputs/outputs of one scoring batch (device pointers).
struct ScoreArgs {
    int64_t n;
    const double* c;      // n*3
    const int32_t* ref;   // n
    double thr;
    double* xy;           // n*2 (projection into ref view, MVS2.py:63)
    uint64_t* mask;       // candidate i's words at mask[i * mstride]
    int32_t* count;       // n (null: records, |V| = popcount of the mask)
    double* avg;          // avg[i * astride] (may be null)
    int32_t* exact_hits;  // 1 counter: lanes that took the exact (numpy-order) path
    int64_t mstride;      // words (separate arrays) or words + 1 (records)
    int64_t astride;      // 1 (separate arrays) or words + 1 (records)
    int rec;              // 1: records [mask words, avg bits] of words + 1 int64 each
};

// Scratch of the tiled scorer (device pointers, sized by the host).
//   tile_count[k * MVS_TC_STRIDE]: tile k's count (stride 1: a wave's atomics
//   on 64 neighbouring tiles share two cache lines -- measured 20 us faster
//   per 2^20 sweep in k_bin than one line per tile, stride 32); then the
//   control block, one 128-B line per counter (their atomics never queue
//   behind each other's): the queue head, fix_count, n_items, done
//   (k_score_fix's finishing ticket) -- tc_words(ntiles) ints
//   sorted[ntiles*cap] = {id, pk} per tile bucket (k_bin writes candidate
//   rank r of tile k at k*cap + r), pk = (x - x0) | (y - y0) << 4 | R << 7
//   (pixel inside the tile); a candidate of rank >= cap overflows to fix_list
//   items = (tile, chunk j, 0, 0): bucket entries [j chunk, (j+1) chunk) of
//   the tile, written in tile order by k_item_scan into segment 0 of
//   kItemSegs (ItemMap presents the segments as one list)
//   fix_list[n], fix_count: {id, tile, pk, 0} of the candidates k_score_fix
//   scores by the direct path -- bucket overflow (k_bin) and candidates with
//   a view decision inside the guard band (the tiled scorers, numpy-order
//   ctNcc there)
#ifndef MVS_TC_STRIDE
#define MVS_TC_STRIDE 1
#endif
constexpr int kTcStride = MVS_TC_STRIDE;
constexpr int kItemSegs = 8;   // k_bin appends work items to 8 segments (workgroup b to segment b % 8)
constexpr int kBandHeads = 8;   // the tiled scorers' band queue heads (one band per XCD)
// one counter set: the tile counts, then the control block: head, fix_count,
// a spare line, the 8 segments' item counts, the band heads (one 128-B line
// each).  Two sets (parities) alternate between batches.
inline int64_t tc_words(int ntiles) { return (int64_t)ntiles * kTcStride + (3 + kItemSegs + kBandHeads) * 32; }

// The per-scene moment tables hold D = n S_bb - S_b^2 (int32) where the
// scorer is k_score_mma_v (V > 64) and w = 1/sqrt(D) (binary64, k_score_tab)
// otherwise.
inline bool moments_dtab(int V) { return V > 64; }

struct TiledArgs {
    int ntx, nty, ntiles;
    int tw, th;                // tile size in pixels (x, y): 16 x 8
    int chunk;                 // candidates per work item
    int cap;                   // bucket capacity per tile (candidates)
    int32_t* tile_count;       // tile k's count at k * kTcStride
    int32_t* head;             // the scorers' work-queue head
    int2* sorted;
    int4* fix_list;
    int32_t* fix_count;
    int32_t* n_items;          // kItemSegs counters, 32 ints apart: items in each segment
    int item_seg;              // capacity of a segment (items of segment x at x * item_seg)
    // the other parity's counter set (tile counts + control block,
    // zero_words ints): the previous batch's, zeroed by this batch's k_bin
    // for the next one
    int32_t* zero_blk;
    int64_t zero_words;
    // view groups of 64 (V > 64: k_score_mma_v scores each work item against
    // every group in turn); groups = 1 otherwise
    int groups;
    // zero_first = 1 asks the launcher to clear both counter sets first (new
    // scratch, or a previous sequence that did not complete)
    int zero_first;
    int4* items;
    // workgroups of the persistent scorer (0: its default, every CU; fewer
    // leave CUs free for a kernel that runs beside it, e.g. RCCL's)
    int grid;
    // implicit items (k_score_tab, dense batches; set by the launcher): item
    // k < ntiles is (tile k, chunk 0) -- tile order without k_item_scan --
    // and k_bin appends the further chunks (tile, j >= 1) to segment 1
    int implicit;
    // direct-path statistics since the context was created (k_score_fix's
    // finishing workgroup; mvs_scorer_stats): [0] candidates on the direct
    // path's list, [1] of them bucket overflow (k_bin), [2] batches
    unsigned long long* stats;
};
// candidates per binning workgroup (k_bin): 1024 threads x MVS_BIN_PER
#ifndef MVS_BIN_PER
#define MVS_BIN_PER 4
#endif
#ifndef MVS_BIN_BLOCK
#define MVS_BIN_BLOCK 1024   // threads per k_bin workgroup (tuning constant)
#endif
#define MVS_BIN_CHUNK (MVS_BIN_BLOCK * MVS_BIN_PER)
// Per-scene window moments of the tiled scorers, one table pair per window
// half-width, built once from the gray stack (k_moments): for pixel (y, x)
// with a valid window and view v, element (y * W + x) * VP + v holds
// S_b = the sum of the signed bytes s = g - 128 over the (2 wid + 1)^2 window
// (int16: |S_b| <= 121 * 128) and
//   V <= 64 (k_score_tab, global table reads): w = 1 / sqrt(n S_bb -
//     S_b^2) (v_rsq_f64 + one Newton step; nan for a constant window and for
//     the pad views V <= v < VP), VP = 16 ceil(V / 16);
//   V > 64 (k_score_mma_v): D = n S_bb - S_b^2 (int32, exact; -1 for the pad
//     views; the scorer forms w from D with the same two instructions),
//     VP = 64 ceil(V / 64).
// The tables hold H W + 16 pixels (a tile row staged whole may run 16 pixels
// past the last one).
struct MomentsDev {
    int16_t* sb;
    double* w;      // V <= 64
    int32_t* d;     // moments_dtab(V): V > 64
    // bit (v & 15) of flat[(y * W + x) * (VP / 16) + v / 16]: view v's window
    // at (x, y) is constant (D = 0) -- 2 B per pixel and 16 views, L2-sized
    // (1.8 MB at dinoRing): k_bin settles candidates with a constant
    // reference window from it
    uint16_t* flat;
    int VP;
    int wid;
};

// One expansion child: (parent record, view v of the parent's V list, i in {-1,+1}).
struct ChildJob {
    int32_t parent;
    int16_t view;
    int16_t di;
};

// Record table (device): one row per scored candidate that may become a patch.
struct RecordsDev {
    double* c;         // 3
    double* n;         // 3
    double* xy;        // 2
    uint64_t* mask;    // words
    int32_t* R;
    int32_t* count;
    uint8_t* color;    // 4 (rgb + pad)
    uint8_t* accept;
    int32_t* cell;     // 2: floor(x/cs), floor(y/cs)
};

struct ExpandArgs {
    int64_t n;                 // children in this launch
    int64_t first_out;         // record index of child 0
    const ChildJob* jobs;
    int cell_size;
    int vlb;
    double dist_thr;           // 0.05 / scale (MVS2.py:369)
    double thr;                // 0.7 (MVS2.py:362)
    int32_t* exact_hits;
};

// Geometry of the tiled scorer (host side sizes scratch with it).
#define MVS_TILE_W 16
#define MVS_TILE_H 8
#define MVS_MMA_CHUNK 1024    // candidates per work item, V <= 64 (whole tiles, as a rule)
#define MVS_GROUP_VIEWS 64    // views per group when V > 64
#define MVS_GROUP_CHUNK 116   // candidates per work item when V > 64 (their reference rows staged)
#ifndef MVS_ACC_PER
#define MVS_ACC_PER 8         // candidates per thread of the exchange's pack (A/B switch)
#endif
#define MVS_ACC_CHUNK (1024 * MVS_ACC_PER)   // candidates per chunk of the exchange's pack (k_acc_pack)

extern "C" {
// RGB -> stack and gv (one pass, coalesced on both sides); the caller zeroes
// both buffers first (pads)
int mvs_launch_build_scene(const SceneDev* sc, const uint8_t* d_rgb, uint8_t* d_stack, uint8_t* d_gv_base,
                           hipStream_t s);
// direct per-candidate scorer (k_score); ev0/ev1 (may be null) are recorded
// on s immediately before and after the kernel
int mvs_launch_score(const SceneDev* sc, const ScoreArgs* a, int wid, hipStream_t s,
                     hipEvent_t ev0, hipEvent_t ev1);
// tiled scorer: k_bin (tile buckets, then the work items), k_score_mma or k_score_mma_v
// (timed by ev0/ev1), k_score_fix
int mvs_launch_score_tiled(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, int wid,
                           const MomentsDev* mt, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
// the window-moment tables of one wid (mvs_score_tab.hip)
int mvs_launch_moments(const SceneDev* sc, const MomentsDev* mt, hipStream_t s);
// k_score_tab (V <= 64, the moments from the tables); k_bin has run
// (V > 64: k_score_mma_v takes the tables through mvs_launch_score_tiled)
int mvs_launch_score_tab(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, const MomentsDev* mt,
                         hipStream_t s);
// dynamic LDS bytes of k_score_mma (0 if the configuration is unsupported)
size_t mvs_mma_lds_bytes(int V, int wid);
// name of the kernel mvs_launch_score / mvs_launch_score_tiled time for (V, wid)
const char* mvs_timed_kernel_name(int V, int wid, int tiled);
// patch_expansion children, one wave each: geometry + direct photo test +
// accept test (small sweeps)
int mvs_launch_expand(const SceneDev* sc, RecordsDev rec, const ExpandArgs* a, int wid,
                      hipStream_t s);
// the same split for large sweeps: geometry (+ colour, projection, cell) of
// every child, then the children's photo test through the tiled scorer, then
// the accept test from the scored counts
int mvs_launch_expand_geom(const SceneDev* sc, RecordsDev rec, const ExpandArgs* a, hipStream_t s);
int mvs_launch_expand_accept(RecordsDev rec, const ExpandArgs* a, hipStream_t s);
// Multi-GPU stage, ingest side: count = popcount(mask) and the accept test
// of children whose masks another rank scored (geometry already in place)
int mvs_launch_expand_ingest(RecordsDev rec, const ExpandArgs* a, int words, hipStream_t s);
// The accepted candidates of a sweep slice as exchange rows [global index,
// mask words, (c != null) x y z bits] after a header row [accepted, n, 0...]
// (each chunk of MVS_ACC_CHUNK candidates in index order, chunks in the order
// they reserve rows), at most cap rows (parallel.PointsExchange), one launch;
// count == null: mask holds records of words + 1 int64 and |V| is their
// popcount; ctl: the pack's counter ([0]) and chunk ticket ([16]), zero
// before the call and left zero after it
int mvs_launch_pack_accepted(int64_t n, int64_t offset, const int32_t* count, const uint64_t* mask, const double* c,
                             int words, int vlb, int64_t cap, unsigned long long* ctl, int64_t* out, hipStream_t s);
// measurement only: a copy of bytes (multiple of 16) by `workgroups` workgroups
int mvs_launch_proxy_copy(void* dst, const void* src, int64_t bytes, int workgroups, hipStream_t s);
int mvs_launch_ncc_windows(int64_t n, int npx, const uint8_t* a, const uint8_t* b, double thr,
                           int force_exact, double* ncc, uint8_t* pass, hipStream_t s);
// stage output order on the device (reconstruct_from_Q, MVS2.py:159-173):
// key[e] = (min view of record events[e]) * nci*ncj + cell x * ncj + cell y,
// or ~0 for an event that is never emitted
int mvs_launch_event_keys(RecordsDev rec, int words, const int32_t* events, int64_t n_events,
                          int nci, int ncj, uint64_t* keys, hipStream_t s);
// rows[i] = [c, rgb] of record idx[i] as float64 (the PLY rows)
int mvs_launch_gather_rows(RecordsDev rec, const int32_t* idx, int64_t n, double* rows, hipStream_t s);
// avg_ncc_score in the reference's arithmetic for records ids[0..n) (ids null:
// records 0..n-1; reads R, xy, mask only) (wid 3 or 5)
int mvs_launch_exact_avg(const SceneDev* sc, RecordsDev rec, int wid, const int32_t* ids, int64_t n,
                         double* out, hipStream_t s);
// stable device sort of (key, value) pairs over the low `bits` key bits;
// tmp == NULL sizes the scratch (*tmp_bytes)
int mvs_sort_pairs(void* tmp, size_t* tmp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                   const int32_t* vals_in, int32_t* vals_out, int64_t n, int bits, hipStream_t s);

// SfM front-end (HarrisFeatures.py, sfm_kernels.hip): Harris response +
// dilate + global max + per-row counts and offsets (rowoff[H] = total), then
// the [col, row] write
int mvs_launch_harris(const SceneDev* sc, int v, double k, float* resp, float* dil, uint32_t* maxkey,
                      int32_t* rowcnt, int32_t* rowoff, hipStream_t s);
int mvs_launch_harris_write(const SceneDev* sc, const float* dil, const uint32_t* maxkey,
                            const int32_t* rowoff, int32_t* out, int64_t cap, hipStream_t s);
int mvs_launch_gather_desc(const SceneDev* sc, int v, const int32_t* rc, int64_t n, int wid,
                           uint32_t* desc, int32_t* S, int32_t* SS, hipStream_t s);
int mvs_launch_match_rows(const uint32_t* dA, const int32_t* SA, const int32_t* SSA, int64_t nA,
                          const uint32_t* dB, const int32_t* SB, const int32_t* SSB, int64_t nB,
                          int npx, double thr, int32_t* best, hipStream_t s);
}

// Internal declarations shared by the HIP kernels (mvs_kernels.hip) and the
// host engine (mvs_engine.cpp).  Not part of the public C-ABI (include/mvs_amd.h).
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

// Window moments of one view at one pixel, 12 bytes: w = 1/sqrt(n S_bb - S_b^2)
// (binary64, 0 for a constant window) and S_b.  S_bb is implied:
// n S_bb - S_b^2 = rint(1/w^2) exactly (db < 2^31, w within 3 ulp).
struct __attribute__((packed, aligned(4))) MomEntry {
    double w;
    uint32_t sb;
};
static_assert(sizeof(MomEntry) == 12, "12-byte moments entries");

// Device-resident scene: the gray stack in quad-interleaved pixel-major
// layout  stack[y][k][v][4] = gray_v(y, 4k..4k+3)  (k = quad index), so that
// one window row of every view is one contiguous run, and one dword holds
// four horizontally adjacent pixels of one view (v_dot4_u32_u8 operand).
struct SceneDev {
    int V, H, W;
    int Wq;            // quads per row, incl. one zero pad quad
    int64_t row_bytes; // Wq * V * 4
    const uint8_t* stack;
    const uint8_t* rgb;      // V*H*W*3 (colour lookups of expansion candidates)
    const CamDev* cams;
    // view-major gray copy gv[v][y][x] (row pitch Wp = W + 16): the reference
    // view's window rows are read with scalar (SMEM) loads
    const uint8_t* gv;
    int Wp;
    // per-view window moments mom[wid][(y*W + x)*V + v] of the (2wid+1)^2
    // window centred at (x, y) (zero where the window is invalid); built once
    // per scene and wid -- the np.mean/np.std ingredients of ctNcc, which do
    // not depend on the reference view
    const struct MomEntry* mom[MVS_MAX_WID + 1];
};

// Inputs/outputs of one scoring batch (device pointers).
struct ScoreArgs {
    int64_t n;
    const double* c;      // n*3
    const int32_t* ref;   // n
    double thr;
    double* xy;           // n*2 (projection into ref view, MVS2.py:63)
    uint64_t* mask;       // n*words
    int32_t* count;       // n
    double* avg;          // n
    int32_t* exact_hits;  // 1 counter: lanes that took the exact (numpy-order) path
};

// Scratch of the tiled scorer (device pointers, sized by the host).
//   tile_count[ntiles+1], tile_off[ntiles+1], item_off[ntiles+1], n_items[1]
//   cand_key[n]  = tile (or -1 if the window is invalid), cand_rank[n],
//   cand_pk[n]   = q | r << 11 | R << 22, sorted[n] = {id, pk} grouped by tile
//   fix_list[n], fix_count[1]: candidates with a view decision inside the guard
//   band, re-scored by k_score_fix (numpy-order ctNcc) after the tiled kernel
struct TiledArgs {
    int ntx, nty, ntiles;
    int tw, th;                // tile size in pixels (x, y): 16x8 tiled kernels, 16x16 MFMA
    int chunk;                 // candidates per work item
    int32_t* tile_count;
    int32_t* tile_off;
    int32_t* item_off;
    int32_t* cand_key;
    int32_t* cand_rank;
    int32_t* cand_pk;
    int2* sorted;
    int32_t* fix_list;
    int32_t* fix_count;
    // view groups (V > 64, k_score_tiledg): work item = (tile chunk, group of
    // 64 views); per (candidate, group) partial count and sum of passing
    // ncc*(n-1), reduced by k_group_finalize.  groups = 1 otherwise.
    int groups;
    int32_t* part_cnt;         // n*groups
    double* part_sum;          // n*groups
    int32_t* xq;               // 8 work-queue heads, one per XCD label (blockIdx % 8)
    // k_tile_scan leaves every counter zero for the next batch (it zeroes the
    // bin counts after reading them and the queue heads / fix_count before the
    // scorer uses them); zero_first = 1 asks the launcher to clear them first
    // (new scratch, or a previous sequence that did not complete)
    int zero_first;
    // work items in the order the scorers take them (k_tile_scan): every full
    // chunk first, then the partial (last) chunks by decreasing size, so the
    // dynamic queues end on the shortest items; int2 = (tile, chunk index)
    int2* items;
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

extern "C" {
int mvs_launch_build_stack(const uint8_t* d_rgb, uint8_t* d_stack, int V, int H, int W, int Wq,
                           hipStream_t s);
// ev0/ev1 (may be null): recorded on s immediately before and after the
// dominant scoring kernel (k_score / k_score_tiled3) -- kernel timing for bench.py
int mvs_launch_score(const SceneDev* sc, const ScoreArgs* a, int wid, hipStream_t s,
                     hipEvent_t ev0, hipEvent_t ev1);
int mvs_launch_build_gv(const uint8_t* d_stack, uint8_t* d_gv, int V, int H, int W, int Wq, int Wp,
                        hipStream_t s);
int mvs_launch_build_moments(const SceneDev* sc, int wid, MomEntry* d_mom, hipStream_t s);
// Tile geometry of the tiled scorers for a W x H image (so the host can size
// scratch): mfma != 0 -> the MFMA scorer's 16x16 tiles, else 16x8.
void mvs_tiled_geometry(int W, int H, int mfma, int* tw, int* th, int* ntx, int* nty);
int mvs_launch_score_tiled(const SceneDev* sc, const ScoreArgs* a, const TiledArgs* t, int wid,
                           int variant, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
int mvs_launch_expand(const SceneDev* sc, RecordsDev rec, const ExpandArgs* a, int wid,
                      hipStream_t s);
// SfM front-end (HarrisFeatures.py): Harris response + dilate + global max +
// per-row counts and offsets (rowoff[H] = total), then the [col, row] write
int mvs_launch_harris(const SceneDev* sc, int v, double k, float* resp, float* dil, uint32_t* maxkey,
                      int32_t* rowcnt, int32_t* rowoff, hipStream_t s);
int mvs_launch_harris_write(const SceneDev* sc, const float* dil, const uint32_t* maxkey,
                            const int32_t* rowoff, int32_t* out, int64_t cap, hipStream_t s);
int mvs_launch_gather_desc(const SceneDev* sc, int v, const int32_t* rc, int64_t n, int wid,
                           uint32_t* desc, int32_t* S, int32_t* SS, hipStream_t s);
int mvs_launch_match_rows(const uint32_t* dA, const int32_t* SA, const int32_t* SSA, int64_t nA,
                          const uint32_t* dB, const int32_t* SB, const int32_t* SSB, int64_t nB,
                          int npx, double thr, int32_t* best, hipStream_t s);
// Packed record rows for the multi-GPU stage exchange: int64 words
// [c0 c1 c2 n0 n1 n2 x y | mask[words] | R + count<<32 | cell0 + cell1<<32 | rgba + accept<<32]
int mvs_launch_pack_records(RecordsDev rec, int words, int64_t first, int64_t n, int64_t* out,
                            hipStream_t s);
int mvs_launch_unpack_records(RecordsDev rec, int words, int64_t first, int64_t n,
                              const int64_t* in, hipStream_t s);
int mvs_launch_ncc_windows(int64_t n, int npx, const uint8_t* a, const uint8_t* b, double thr,
                           int force_exact, double* ncc, uint8_t* pass, hipStream_t s);
}

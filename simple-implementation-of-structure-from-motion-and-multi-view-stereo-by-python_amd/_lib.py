"""ctypes binding of libmvs_amd.so (include/mvs_amd.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises RuntimeError (the one exception the
reference's main() catches, main.py:43-46).
"""
import atexit
import ctypes
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmvs_amd.so")

_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p

# (name, restype, argtypes) -- mirrors include/mvs_amd.h one to one
SIGNATURES = [
    ("mvs_version", ctypes.c_char_p, []),
    ("mvs_last_error", ctypes.c_char_p, [_vp]),
    ("mvs_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p,
                                      _dp, _dp, _dp, _dp, ctypes.POINTER(_vp)]),
    ("mvs_ctx_destroy", None, [_vp]),
    ("mvs_ctx_rproj", ctypes.c_int, [_vp, _dp]),
    ("mvs_ctx_rebuild", ctypes.c_int, [_vp, _vp]),
    ("mvs_score", ctypes.c_int, [_vp, ctypes.c_int64, _dp, _i32p, ctypes.c_int, ctypes.c_double,
                                 _dp, _u64p, _i32p, _dp]),
    ("mvs_score_device", ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, ctypes.c_int,
                                        ctypes.c_double, _vp, _vp, _vp, _vp, _vp]),
    ("mvs_score_device_rec", ctypes.c_int, [_vp, ctypes.c_int64, _vp, _vp, ctypes.c_int, ctypes.c_double,
                                            _vp, _vp, _vp]),
    ("mvs_pack_accepted", ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int,
                                         ctypes.c_int64, _vp, _vp]),
    ("mvs_set_scorer_grid", ctypes.c_int, [_vp, ctypes.c_int]),
    ("mvs_proxy_copy", ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp]),
    ("mvs_filter_outliers", ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p,
                                           _u64p, _i32p, _dp, _dp, _dp, _u8p, _i64p]),
    ("mvs_exact_hits", ctypes.c_int64, [_vp]),
    ("mvs_scorer_stats", ctypes.c_int, [_vp, _i64p]),
    ("mvs_stream_retiring", ctypes.c_int, [_vp, _vp]),
    ("mvs_kernel_timing", ctypes.c_int, [_vp, ctypes.c_int]),
    ("mvs_kernel_time", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_int64)]),
    ("mvs_timed_kernel", ctypes.c_char_p, [_vp]),
    ("mvs_ncc_windows", ctypes.c_int, [ctypes.c_int64, ctypes.c_int, _vp, _vp, ctypes.c_double,
                                       ctypes.c_int, _vp, _vp, _vp]),
    ("mvs_stage_run", ctypes.c_int, [_vp, ctypes.c_int64, _i64p, _i32p, _fp, ctypes.c_int,
                                     ctypes.c_double, ctypes.c_int, ctypes.c_int64,
                                     ctypes.POINTER(_vp)]),
    ("mvs_stage_begin", ctypes.c_int, [_vp, ctypes.c_int64, _i64p, _i32p, _fp, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(_vp)]),
    ("mvs_stage_plan", ctypes.c_int64, [_vp]),
    ("mvs_stage_record_width", ctypes.c_int, [_vp]),
    ("mvs_stage_score_slice", ctypes.c_int, [_vp, _vp]),
    ("mvs_stage_ingest", ctypes.c_int, [_vp, _vp]),
    ("mvs_stage_finish", ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    ("mvs_stage_destroy", None, [_vp]),
    ("mvs_stage_count", ctypes.c_int64, [_vp, ctypes.c_int]),
    ("mvs_stage_rows", ctypes.c_int, [_vp, ctypes.c_int, _dp]),
    ("mvs_stage_rows_device", ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp]),
    ("mvs_stage_stats", ctypes.c_int, [_vp, _i64p]),
    ("mvs_stage_times", ctypes.c_int, [_vp, _dp]),
    ("mvs_stage_set_options", ctypes.c_int, [_vp, ctypes.c_int]),
    ("mvs_exact_avg", ctypes.c_int, [_vp, ctypes.c_int64, _i32p, _dp, _u64p, ctypes.c_int, _dp]),
    ("mvs_stage_filter_stats", ctypes.c_int, [_vp, _i64p]),
    ("mvs_stage_free", None, [_vp]),
    ("mvs_expand_candidates", ctypes.c_int, [_vp, ctypes.c_int64, _dp, _dp, _dp, ctypes.c_int64,
                                             _i32p, _i32p, _i32p, ctypes.c_int, ctypes.c_double,
                                             ctypes.c_int, ctypes.c_double, _dp, _dp, _u8p, _dp,
                                             _u64p, _i32p, _u8p]),
    ("mvs_rodrigues_roundtrip", ctypes.c_int, [_dp, _dp]),
    ("mvs_triangulate", ctypes.c_int, [_dp, _dp, _dp, _dp, _dp]),
    ("mvs_harris_points", ctypes.c_int, [_vp, ctypes.c_int, _i32p, ctypes.c_int64, _i64p]),
    ("mvs_match_two_sided", ctypes.c_int, [_vp, ctypes.c_int, _i32p, ctypes.c_int64, ctypes.c_int,
                                           _i32p, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                           _i32p, _i32p, _i32p]),
    ("mvs_sfm_pair", ctypes.c_int, [_dp, _dp, _dp, _dp, _dp, _dp, ctypes.c_int64, _fp, _fp,
                                    ctypes.c_double, _fp, _u8p]),
]

_lib = None


def load(path=None):
    """Load libmvs_amd.so; raises RuntimeError if it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("MVS_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise RuntimeError(
            f"libmvs_amd.so not found at {path}: build it with __graft_entry__.build() "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # torch first: its bundled HIP runtime (SONAME libamdhip64.so.7) is then
    # the one libmvs_amd.so's NEEDED entry binds to, so torch tensors, torch
    # streams and the library share one runtime.  Loaded the other way round
    # the process would hold two HIP runtimes and torch.cuda would not start.
    import torch  # noqa: F401
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        raise RuntimeError(f"cannot load {path}: {e}") from e
    for name, res, args in SIGNATURES:
        if path != LIB_PATH and not hasattr(lib, name):
            continue   # an older A/B build (MVS_LIB) without a newer entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a, t):
    return a.ctypes.data_as(t)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def last_error(ctx=None):
    msg = load().mvs_last_error(ctx)
    return msg.decode() if msg else ""


MVS_E_DIVZERO = -5
MVS_STAGE_FILTER_OUTLIERS = 1


def check(rc, ctx=None, what="mvs"):
    if rc == MVS_E_DIVZERO:
        # where the reference itself raises (filter_out_outlier, MVS2.py:144)
        raise ZeroDivisionError(f"{what}: {last_error(ctx)}")
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error(ctx)}")


def rodrigues_roundtrip(R):
    """R' = Rodrigues(Rodrigues(R)) -- the rotation cv2.projectPoints applies (utils.py:242-243)."""
    R = _c(R, np.float64).reshape(9)
    out = np.empty(9)
    check(load().mvs_rodrigues_roundtrip(_p(R, _dp), _p(out, _dp)), what="rodrigues")
    return out.reshape(3, 3)


def sfm_pair(KA, RA, tA, KB, RB, tB, q, tr, max_err):
    """One pair of StructureFromMotion's loop (SFM.py:60-80), host C++:
    (float32 points (n, 3), keep (n,) bool)."""
    mats = [_c(m, np.float64).reshape(-1) for m in (KA, RA, tA, KB, RB, tB)]
    q = _c(q, np.float32).reshape(-1, 2)
    tr = _c(tr, np.float32).reshape(-1, 2)
    n = len(q)
    if len(tr) != n:
        raise RuntimeError("query and train correspondences differ in length")
    pt = np.empty((max(n, 1), 3), np.float32)
    keep = np.empty(max(n, 1), np.uint8)
    check(load().mvs_sfm_pair(*[_p(m, _dp) for m in mats], n, _p(q, _fp), _p(tr, _fp),
                              float(max_err), _p(pt, _fp), _p(keep, _u8p)), None, "mvs_sfm_pair")
    return pt[:n], keep[:n].astype(bool)


def filter_outliers(cell, mask, count, avg, c, nrm, nci, ncj):
    """CellTable.filter_out_outlier (MVS2.py:132-158) on the host over accepted
    patches in fill order (mvs_filter_outliers): -> (alive bool (n,), removed,
    "remove a outlier" lines).  Raises ZeroDivisionError where the reference does."""
    cell = _c(cell, np.int32).reshape(-1, 2)
    n = len(cell)
    mask = _c(mask, np.uint64).reshape(n, -1)
    count = _c(count, np.int32).reshape(n)
    avg = _c(avg, np.float64).reshape(n)
    c = _c(c, np.float64).reshape(n, 3)
    nrm = _c(nrm, np.float64).reshape(n, 3)
    alive = np.empty(max(n, 1), np.uint8)
    stats = np.zeros(2, np.int64)
    check(load().mvs_filter_outliers(n, mask.shape[1], int(nci), int(ncj), _p(cell, _i32p), _p(mask, _u64p),
                                     _p(count, _i32p), _p(avg, _dp), _p(c, _dp), _p(nrm, _dp),
                                     _p(alive, _u8p), _p(stats, _i64p)), None, "mvs_filter_outliers")
    return alive[:n].astype(bool), int(stats[0]), int(stats[1])


def triangulate(P1, P2, x1, x2):
    """cv2.triangulatePoints for one correspondence (utils.py:238-239), homogeneous 4-vector."""
    P1 = _c(P1, np.float64).reshape(12)
    P2 = _c(P2, np.float64).reshape(12)
    x1 = _c(x1, np.float64).reshape(2)
    x2 = _c(x2, np.float64).reshape(2)
    out = np.empty(4)
    check(load().mvs_triangulate(_p(P1, _dp), _p(P2, _dp), _p(x1, _dp), _p(x2, _dp), _p(out, _dp)),
          what="triangulate")
    return out


# live contexts: a retiring caller stream is announced to each of them
# (stream_retiring), and the ones still open at interpreter exit are closed by
# an atexit hook, before the HIP runtime's own teardown
_LIVE = weakref.WeakSet()


def stream_retiring(stream):
    """A caller stream (a hipStream_t handle) is about to be destroyed: every
    live context waits for its work there now (mvs_stream_retiring)."""
    for cx in list(_LIVE):
        h = getattr(cx, "_h", None)
        if h:
            check(load().mvs_stream_retiring(h, stream), h, "mvs_stream_retiring")


@atexit.register
def _close_live_contexts():
    for cx in list(_LIVE):
        try:
            cx.close()
        except Exception:
            pass


class MvsContext:
    """One device-resident scene (images + cameras) on one GPU.

    imgs: (V,H,W,3) uint8 RGB (main.py:17-18 convention) or a list of such
    frames; K, R: (V,3,3); t: (V,3) or (V,3,1).
    """

    def __init__(self, imgs, K, R, t, device=0, Rp=None):
        lib = load()
        rgb = _c(np.stack(imgs) if isinstance(imgs, (list, tuple)) else imgs, np.uint8)
        if rgb.ndim != 4 or rgb.shape[-1] != 3:
            raise RuntimeError(f"images must be (V,H,W,3) uint8 RGB, got {rgb.shape}")
        self.V, self.H, self.W = (int(x) for x in rgb.shape[:3])
        self.words = (self.V + 63) // 64
        K = _c(K, np.float64).reshape(self.V, 9)
        R = _c(R, np.float64).reshape(self.V, 9)
        t = _c(t, np.float64).reshape(self.V, 3)
        rp = _c(Rp, np.float64).reshape(self.V, 9) if Rp is not None else None
        h = _vp()
        rc = lib.mvs_ctx_create(int(device), self.V, self.H, self.W, _p(rgb, _u8p), _p(K, _dp),
                                _p(R, _dp), _p(t, _dp), _p(rp, _dp) if rp is not None else None,
                                ctypes.byref(h))
        check(rc, None, "mvs_ctx_create")
        self._h = h
        self.device = device
        self._stages = weakref.WeakSet()
        _LIVE.add(self)

    def close(self):
        if getattr(self, "_h", None):
            # stepped stages hold the context: they go first
            for st in list(getattr(self, "_stages", ())):
                st.close()
            load().mvs_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def rproj(self):
        out = np.empty((self.V, 9))
        check(load().mvs_ctx_rproj(self._h, _p(out, _dp)), self._h, "mvs_ctx_rproj")
        return out.reshape(self.V, 3, 3)

    def exact_hits(self):
        return int(load().mvs_exact_hits(self._h))

    def scorer_stats(self):
        """{'direct': candidates the direct path re-scored (guard band +
        bucket overflow), 'overflow': of them bucket overflow, 'batches':
        tiled batches} since the context was created (mvs_scorer_stats)."""
        out = np.zeros(3, np.int64)
        check(load().mvs_scorer_stats(self._h, _p(out, _i64p)), self._h, "mvs_scorer_stats")
        return {"direct": int(out[0]), "overflow": int(out[1]), "batches": int(out[2])}

    def rebuild(self, stream=None):
        """Rebuild the device gray stack / view-major copy from the resident
        RGB images (stream-ordered; for cold-sweep timing)."""
        check(load().mvs_ctx_rebuild(self._h, stream), self._h, "mvs_ctx_rebuild")

    def kernel_timing(self, enable=True, every=1):
        """Start (reset) or stop HIP-event timing of the dominant scoring kernel;
        every = k times every k-th scoring call."""
        check(load().mvs_kernel_timing(self._h, int(every) if enable else 0), self._h, "mvs_kernel_timing")

    def kernel_time(self):
        """-> (total kernel milliseconds, timed launches) since kernel_timing(True)."""
        ms = ctypes.c_double(0.0)
        k = ctypes.c_int64(0)
        check(load().mvs_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(k)), self._h,
              "mvs_kernel_time")
        return ms.value, int(k.value)

    def timed_kernel(self):
        """Name of the kernel the last timed event pair bracketed."""
        name = load().mvs_timed_kernel(self._h)
        return name.decode() if name else ""

    def score(self, c, ref, min_ncc=0.7, wid=5):
        """Batched photo_consistenecy_test (MVS2.py:62-77) on host arrays.

        Returns xy (n,2), mask (n,words) uint64, count (n,), avg (n,)."""
        c = _c(c, np.float64).reshape(-1, 3)
        ref = _c(ref, np.int32).reshape(-1)
        n = len(ref)
        if len(c) != n:
            raise RuntimeError("c and ref lengths differ")
        xy = np.empty((n, 2))
        mask = np.empty((n, self.words), np.uint64)
        count = np.empty(n, np.int32)
        avg = np.empty(n)
        rc = load().mvs_score(self._h, n, _p(c, _dp), _p(ref, _i32p), int(wid), float(min_ncc),
                              _p(xy, _dp), _p(mask, _u64p), _p(count, _i32p), _p(avg, _dp))
        check(rc, self._h, "mvs_score")
        return xy, mask, count, avg

    def exact_avg(self, ref, xy, mask, wid=5):
        """avg_ncc_score in the reference's arithmetic (numpy-order ctNcc, summed in
        view order) for candidates scored by `score`: bit-exact, where score's avg
        is within 1e-12."""
        ref = _c(ref, np.int32).reshape(-1)
        n = len(ref)
        xy = _c(xy, np.float64).reshape(n, 2)
        mask = _c(mask, np.uint64).reshape(n, self.words)
        out = np.empty(n)
        check(load().mvs_exact_avg(self._h, n, _p(ref, _i32p), _p(xy, _dp), _p(mask, _u64p), int(wid),
                                   _p(out, _dp)), self._h, "mvs_exact_avg")
        return out

    def score_device(self, c, ref, xy, mask, count, avg, min_ncc=0.7, wid=5, stream=None):
        """Same on device tensors (torch: pass .data_ptr() ints); stream-ordered."""
        n = int(ref.numel()) if hasattr(ref, "numel") else int(len(ref))
        ptr = (lambda x: x.data_ptr()) if hasattr(ref, "data_ptr") else (lambda x: int(x))
        rc = load().mvs_score_device(self._h, n, ptr(c), ptr(ref), int(wid), float(min_ncc),
                                     ptr(xy), ptr(mask), ptr(count),
                                     ptr(avg) if avg is not None else None,
                                     stream if stream is not None else None)
        check(rc, self._h, "mvs_score_device")

    def score_device_rec(self, c, ref, xy, rec, min_ncc=0.7, wid=5, stream=None):
        """The photo test into records (device int64 tensor (n, words + 1): mask
        words, avg bits; |V| = popcount), stream-ordered."""
        n = int(ref.numel())
        if rec.dtype.itemsize != 8 or tuple(rec.shape) != (n, self.words + 1) or not rec.is_contiguous():
            raise RuntimeError(f"score_device_rec: rec must be contiguous int64 ({n}, {self.words + 1})")
        rc = load().mvs_score_device_rec(self._h, n, c.data_ptr(), ref.data_ptr(), int(wid), float(min_ncc),
                                         xy.data_ptr(), rec.data_ptr(), stream if stream is not None else None)
        check(rc, self._h, "mvs_score_device_rec")

    def pack_accepted(self, offset, count, mask, vlb, out, stream=None, c=None):
        """mvs_pack_accepted: the accepted candidates (count >= vlb) of a scored
        slice as exchange rows of out (device int64 tensor (cap + 1, width):
        row 0 = [accepted, n, 0...], then rows
        [offset + i, mask words(, x y z bits with c)]: each 8,192-candidate
        chunk in index order, the chunks in any order -- sort_rows() orders
        them); c = the
        slice's (n, 3) float64 centres or None (width 1 + words [+ 3]);
        stream-ordered, no host sync.  count None: mask is score_device_rec's
        records and |V| their popcount."""
        n = int(count.numel()) if count is not None else int(mask.shape[0])
        # the kernel indexes rows at a fixed pitch: strided views would give wrong rows
        if count is None and (mask.dtype.itemsize != 8 or mask.dim() != 2 or mask.shape[1] != self.words + 1
                              or not mask.is_contiguous()):
            raise RuntimeError("pack_accepted: records must be contiguous int64 (n, words + 1)")
        if count is not None and (count.dtype.itemsize != 4 or not count.is_contiguous()
                                  or mask.dtype.itemsize != 8 or tuple(mask.shape) != (n, self.words)
                                  or not mask.is_contiguous()):
            raise RuntimeError(f"pack_accepted: count must be contiguous int32 (n,) and mask contiguous "
                               f"int64 (n, {self.words})")
        cap = int(out.shape[0]) - 1
        width = 1 + self.words + (3 if c is not None else 0)
        if out.dtype.itemsize != 8 or out.shape[1] != width or not out.is_contiguous():
            raise RuntimeError(f"pack_accepted: out must be contiguous int64 (cap + 1, {width})")
        if c is not None and (c.dtype.itemsize != 8 or tuple(c.shape) != (n, 3) or not c.is_contiguous()):
            raise RuntimeError("pack_accepted: c must be contiguous float64 (n, 3)")
        rc = load().mvs_pack_accepted(self._h, n, int(offset), count.data_ptr() if count is not None else None,
                                      mask.data_ptr(),
                                      c.data_ptr() if c is not None else None,
                                      int(vlb), cap, out.data_ptr(),
                                      stream if stream is not None else None)
        check(rc, self._h, "mvs_pack_accepted")

    def set_scorer_grid(self, workgroups=0):
        """Hold the persistent scorers to `workgroups` workgroups (0: default,
        two per CU): the grid for a CU-masked scoring stream."""
        check(load().mvs_set_scorer_grid(self._h, int(workgroups)), self._h, "mvs_set_scorer_grid")

    def harris_points(self, view):
        """getHarrisPoints(imgs[view]) (HarrisFeatures.py:135-161) on the GPU:
        int32 (n, 2) [col, row] in np.where's row-major order."""
        lib = load()
        n = ctypes.c_int64(0)
        check(lib.mvs_harris_points(self._h, int(view), None, 0, ctypes.byref(n)), self._h,
              "mvs_harris_points")
        out = np.empty((max(n.value, 1), 2), np.int32)
        check(lib.mvs_harris_points(self._h, int(view), _p(out, _i32p), n.value, ctypes.byref(n)),
              self._h, "mvs_harris_points")
        return out[:n.value]

    def match_two_sided(self, view_a, pts_a, view_b, pts_b, thr=0.5, wid=5):
        """MatchTwoSided over getDescFeatures windows (HarrisFeatures.py:15-67) on the
        GPU; pts_* [row, col] inside getDescFeatures' bounds.
        Returns (m12, best12, best21) int32 (-1 = none)."""
        a = _c(pts_a, np.int32).reshape(-1, 2)
        b = _c(pts_b, np.int32).reshape(-1, 2)
        m12 = np.empty(max(len(a), 1), np.int32)
        b12 = np.empty(max(len(a), 1), np.int32)
        b21 = np.empty(max(len(b), 1), np.int32)
        check(load().mvs_match_two_sided(self._h, int(view_a), _p(a, _i32p), len(a), int(view_b),
                                         _p(b, _i32p), len(b), int(wid), float(thr), _p(m12, _i32p),
                                         _p(b12, _i32p), _p(b21, _i32p)),
              self._h, "mvs_match_two_sided")
        return m12[:len(a)], b12[:len(a)], b21[:len(b)]

    def expand_candidates(self, pc, pn, pxy, job_parent, job_view, job_di, cell_size=2,
                          scale=10.0, wid=5, min_ncc=0.7):
        """patch_expansion candidates (MVS2.py:329-369) for explicit jobs (see mvs_amd.h)."""
        pc = _c(pc, np.float64).reshape(-1, 3)
        pn = _c(pn, np.float64).reshape(-1, 3)
        pxy = _c(pxy, np.float64).reshape(-1, 2)
        jp = _c(job_parent, np.int32)
        jv = _c(job_view, np.int32)
        jd = _c(job_di, np.int32)
        n = len(jp)
        X, nX, xy = np.empty((n, 3)), np.empty((n, 3)), np.empty((n, 2))
        color = np.empty((n, 3), np.uint8)
        mask = np.empty((n, self.words), np.uint64)
        count = np.empty(n, np.int32)
        acc = np.empty(n, np.uint8)
        rc = load().mvs_expand_candidates(self._h, len(pc), _p(pc, _dp), _p(pn, _dp), _p(pxy, _dp),
                                          n, _p(jp, _i32p), _p(jv, _i32p), _p(jd, _i32p),
                                          int(cell_size), float(scale), int(wid), float(min_ncc),
                                          _p(X, _dp), _p(nX, _dp), _p(color, _u8p), _p(xy, _dp),
                                          _p(mask, _u64p), _p(count, _i32p), _p(acc, _u8p))
        check(rc, self._h, "mvs_expand_candidates")
        return X, nX, color, xy, mask, count, acc

    def stage(self, track_off, obs_view, obs_xy, cell_size=2, scale=1.0, wid=5, max_pops=100000,
              filter_outliers=False):
        """DensePointsWithMVS2 minus IO; returns (initial N0x6, all Nx6, stats dict).
        filter_outliers: run CellTable.filter_out_outlier (MVS2.py:132-158) before
        the reconstruction, as if MVS2.py:281 were enabled."""
        lib = load()
        track_off, obs_view, obs_xy = _tracks(track_off, obs_view, obs_xy)
        self.set_stage_options(filter_outliers)
        res = _vp()
        rc = lib.mvs_stage_run(self._h, len(track_off) - 1, _p(track_off, _i64p),
                               _p(obs_view, _i32p), _p(obs_xy, _fp), int(cell_size), float(scale),
                               int(wid), int(max_pops), ctypes.byref(res))
        check(rc, self._h, "mvs_stage_run")
        return _take_result(res, self._h)

    def set_stage_options(self, filter_outliers=False):
        """Options of the stage runs that follow (mvs_stage_set_options)."""
        flags = MVS_STAGE_FILTER_OUTLIERS if filter_outliers else 0
        check(load().mvs_stage_set_options(self._h, flags), self._h, "mvs_stage_set_options")

    def stage_begin(self, track_off, obs_view, obs_xy, cell_size=2, scale=1.0, wid=5,
                    max_pops=100000, rank=0, world=1):
        """The stage in steps (mvs_stage_begin ...); see parallel.stage_sharded."""
        return Stage(self, track_off, obs_view, obs_xy, cell_size, scale, wid, max_pops, rank, world)


STAGE_STATS = ["pops", "tests", "accepts", "queue_left", "scored", "sweeps", "seed_candidates",
               "exact_hits"]
STAGE_TIMES = ["seed_s", "commit_s", "gpu_sweeps_s", "copy_back_s", "output_s", "total_s"]
# + "rows_to_host_s": the copy of the PLY rows from HBM into the numpy arrays


def _tracks(track_off, obs_view, obs_xy):
    return (_c(track_off, np.int64), _c(obs_view, np.int32),
            _c(obs_xy, np.float32).reshape(-1, 2))


def _take_result(res, h):
    """Copy an mvs_stage_result out and free it -> (initial, all, stats)."""
    import time
    lib = load()
    try:
        t0 = time.perf_counter()
        out = []
        for which in (0, 1):
            n = lib.mvs_stage_count(res, which)
            rows = np.empty((n, 6))
            if n:
                check(lib.mvs_stage_rows(res, which, _p(rows, _dp)), h, "mvs_stage_rows")
            out.append(rows)
        t_rows = time.perf_counter() - t0
        st = np.empty(8, np.int64)
        check(lib.mvs_stage_stats(res, _p(st, _i64p)), h, "mvs_stage_stats")
        tm = np.empty(6)
        check(lib.mvs_stage_times(res, _p(tm, _dp)), h, "mvs_stage_times")
        fl = np.empty(2, np.int64)
        check(lib.mvs_stage_filter_stats(res, _p(fl, _i64p)), h, "mvs_stage_filter_stats")
    finally:
        lib.mvs_stage_free(res)
    stats = dict(zip(STAGE_STATS, (int(x) for x in st)))
    stats["times"] = dict(zip(STAGE_TIMES, (float(x) for x in tm)))
    stats["times"]["rows_to_host_s"] = t_rows
    stats["outliers_removed"], stats["outlier_lines"] = int(fl[0]), int(fl[1])
    return out[0], out[1], stats


class Stage:
    """One rank's view of a stepped stage run (include/mvs_amd.h, mvs_stage_*)."""

    def __init__(self, ctx, track_off, obs_view, obs_xy, cell_size, scale, wid, max_pops, rank,
                 world):
        lib = load()
        self.ctx = ctx
        self.rank, self.world = int(rank), int(world)
        self._tr = _tracks(track_off, obs_view, obs_xy)
        h = _vp()
        rc = lib.mvs_stage_begin(ctx.handle, len(self._tr[0]) - 1, _p(self._tr[0], _i64p),
                                 _p(self._tr[1], _i32p), _p(self._tr[2], _fp), int(cell_size),
                                 float(scale), int(wid), int(max_pops), self.rank, self.world,
                                 ctypes.byref(h))
        check(rc, ctx.handle, "mvs_stage_begin")
        self._st = h
        self.width = lib.mvs_stage_record_width(h)
        ctx._stages.add(self)   # closed before their context (MvsContext.close)

    def plan(self):
        """Commit and plan the next sweep -> its job count (0: finished)."""
        n = load().mvs_stage_plan(self._st)
        if n < 0:
            check(int(n), self.ctx.handle, "mvs_stage_plan")
        return int(n)

    def slice_max(self, nj):
        return -(-nj // self.world)

    def score_slice(self, out=None):
        """Score this rank's slice; out = device int64 tensor (slice_max, width) when world > 1."""
        ptr = out.data_ptr() if out is not None else None
        check(load().mvs_stage_score_slice(self._st, ptr), self.ctx.handle, "mvs_stage_score_slice")

    def ingest(self, gathered=None):
        """gathered = device int64 tensor (world, slice_max, width) when world > 1.

        The library reads it on its own stream, which does not wait for torch's:
        the producer (all-gather, torch.stack) is synchronised here first."""
        if gathered is not None and getattr(gathered, "is_cuda", False):
            import torch
            torch.cuda.current_stream(gathered.device).synchronize()
        ptr = gathered.data_ptr() if gathered is not None else None
        check(load().mvs_stage_ingest(self._st, ptr), self.ctx.handle, "mvs_stage_ingest")

    def finish(self):
        res = _vp()
        check(load().mvs_stage_finish(self._st, ctypes.byref(res)), self.ctx.handle, "mvs_stage_finish")
        return _take_result(res, self.ctx.handle)

    def close(self):
        if self._st:
            load().mvs_stage_destroy(self._st)
            self._st = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def proxy_copy(dst, src, nbytes, workgroups, stream=None):
    """Measurement only: copy nbytes between device tensors with a kernel of
    `workgroups` workgroups on `stream` (a collective's CU footprint)."""
    check(load().mvs_proxy_copy(dst.data_ptr(), src.data_ptr(), int(nbytes), int(workgroups), stream),
          None, "mvs_proxy_copy")


def ncc_windows(a, b, thr, force_exact=False, stream=None):
    """ctNcc on device window pairs (torch uint8 tensors (n, npx)); returns (ncc, pass) tensors."""
    import torch
    n, npx = a.shape
    ncc = torch.empty(n, dtype=torch.float64, device=a.device)
    ok = torch.empty(n, dtype=torch.uint8, device=a.device)
    rc = load().mvs_ncc_windows(n, npx, a.data_ptr(), b.data_ptr(), float(thr), int(force_exact),
                                ncc.data_ptr(), ok.data_ptr(), stream)
    check(rc, None, "mvs_ncc_windows")
    return ncc, ok

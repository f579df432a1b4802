"""SfM front-end: the producer of the MVS stage's seed tracks.

The reference builds its tracks in SFM.StructureFromMotion (SFM.py:47-88):
for every consecutive image pair it gets correspondences (getORBFeatures:
OpenCV ORB + FLANN + RANSAC, utils.py:160-232), triangulates them with the
known cameras, drops points whose reprojection error exceeds
MIN_REPROJECTION_ERROR and merges the rest into a GlobalSet (GlobalSet.py),
whose legal sets' point2d_list are what DensePointsWithMVS2 seeds from.

Here:
  GlobalSet / MySet        the track store with GlobalSet.py's semantics,
                           including the point2d_list order its set unions
                           produce (element 0 is the MVS reference view)
  StructureFromMotion      SFM.py:47-88 with a pluggable correspondence source;
                           the pair geometry (triangulation, float32 point,
                           reprojection test) is mvs_sfm_pair (host C++)
  harris_matches           the correspondence source that runs here
                           (BASELINE config 5): getHarrisPoints +
                           getDescFeatures + MatchTwoSided + getMatches
                           (HarrisFeatures.py) with the Harris map and the
                           all-pairs NCC matching on the GPU
                           (mvs_harris_points, mvs_match_two_sided)

OpenCV's ORB/FLANN/RANSAC is not available in this image and is not
reproduced.  Bundle adjustment (DrawPointClouds, SFM.py:91-228) only moves
world points, which the MVS stage never reads; it is not run.
"""
import math

import numpy as np

from . import _lib
from .utils import pars_to_arrays, read_pars


class MySet(object):
    """One track: world point + observations (GlobalSet.py:5-20)."""

    def __init__(self, world_point, point2d_list):
        self.world_point = world_point
        self.point2d_list = point2d_list

    def union(self, other_world_point, other_point2d_list):
        # the observation list becomes the set union's iteration order
        self.point2d_list = list(set(self.point2d_list) | set(other_point2d_list))

    def union_with(self, other):
        self.point2d_list = list(set(self.point2d_list) | set(other.point2d_list))


class GlobalSet(object):
    """Tracks keyed by their (view, x, y) observations (GlobalSet.py:22-175).

    add2pts(a_list, point): a_list = [(view_a, x, y), (view_b, x, y)] of one
    triangulated correspondence.  An observation seen before joins its set if
    the new point is within `threshold` of the set's world point; two known
    observations of different sets merge those sets; otherwise the sets
    involved are invalidated.  getInfo() -> (n_observations, n_points3d,
    legal sets in creation order)."""

    def __init__(self, threshold=0.01):
        self.threshold = threshold
        self.valid = {}
        self.set_list = {}
        self.set_index = {}
        self.list_ct = 0

    def clear(self):
        self.valid.clear()
        self.set_list.clear()
        self.set_index.clear()
        self.list_ct = 0

    def getInfo(self):
        legal = [s for k, s in self.set_list.items() if self.valid[k]]
        return sum(len(s.point2d_list) for s in legal), len(legal), legal

    def updateWorldPoints(self, update_world_pt):
        it = iter(update_world_pt)
        for k, s in self.set_list.items():
            if self.valid[k]:
                s.world_point = next(it).world_point

    def show_list(self):
        for s in self.set_list.values():
            print(s.world_point, s.point2d_list)

    def check_threshold(self, set_idx, b):
        # elementwise arithmetic in the points' own dtype (float32), sqrt in double
        a = self.set_list[set_idx].world_point
        return math.sqrt((a[0] - b[0]) ** 2 + (a[1] - b[1]) ** 2 + (a[2] - b[2]) ** 2) < self.threshold

    def _joins(self, idx, point):
        return self.valid[idx] and self.check_threshold(idx, point)

    def add2pts(self, a_list, a_3d_point):
        first, second = a_list[0], a_list[1]
        i1 = self.set_index.get(first, -1)
        i2 = self.set_index.get(second, -1)
        if i1 == -1 and i2 == -1:
            k = self.list_ct
            self.set_index[first] = k
            self.set_index[second] = k
            self.set_list[k] = MySet(a_3d_point, a_list)
            self.valid[k] = True
            self.list_ct += 1
        elif i1 == -1 or i2 == -1:
            known, new = (i2, first) if i1 == -1 else (i1, second)
            if self._joins(known, a_3d_point):
                self.set_index[new] = known
                self.set_list[known].union(a_3d_point, a_list)
            else:
                self.valid[known] = False
        elif i1 == i2:
            if self._joins(i1, a_3d_point):
                self.set_list[i1].union(a_3d_point, a_list)
            else:
                self.valid[i2] = False
        elif self.valid[i1] and self.valid[i2] and self.check_threshold(i1, a_3d_point):
            self.set_list[i1].union_with(self.set_list[i2])
            for ob in self.set_list[i2].point2d_list:
                self.set_index[ob] = i1
            del self.set_list[i2]
        else:
            self.valid[i2] = False
            self.valid[i1] = False


def sequence_pairs(n_images):
    """getSequence (utils.py:101-113): consecutive pairs (i-1, i)."""
    return [(i - 1, i) for i in range(1, n_images)]


def desc_bounds_rc(pts_cr, H, W, wid=5):
    """[col, row] points -> the [row, col] ones getDescFeatures keeps
    (HarrisFeatures.py:128), in order."""
    p = np.asarray(pts_cr, np.int64).reshape(-1, 2)
    r, c = p[:, 1], p[:, 0]
    ok = (r - wid >= 0) & (r + wid + 1 < H) & (c - wid > 0) & (c + wid + 1 < W)
    return np.stack([r[ok], c[ok]], 1).astype(np.int32)


def get_matches(locs1, locs2, m12):
    """getMatches(..., show_below=False) (HarrisFeatures.py:82-114): pairs with
    m > 0 (index 0 never matches there), [row, col] -> [col, row] int32."""
    m12 = np.asarray(m12)
    i = np.nonzero(m12 > 0)[0]
    src = np.asarray(locs1)[i][:, ::-1]
    dst = np.asarray(locs2)[m12[i]][:, ::-1]
    return (np.ascontiguousarray(src, np.int32).reshape(-1, 2),
            np.ascontiguousarray(dst, np.int32).reshape(-1, 2))


class HarrisMatcher:
    """Correspondences of an image pair from the reference's Harris/NCC
    features, on the GPU: getHarrisPoints per view (cached), the points
    getDescFeatures keeps, MatchTwoSided(thr 0.5), getMatches; returned like
    getORBFeatures: (query float32 (n, 2), train float32 (n, 2), n)."""

    def __init__(self, ctx, wid=5, thr=0.5):
        self.ctx, self.wid, self.thr = ctx, wid, thr
        self._locs = {}

    def locs(self, view):
        if view not in self._locs:
            self._locs[view] = desc_bounds_rc(self.ctx.harris_points(view), self.ctx.H, self.ctx.W,
                                              self.wid)
        return self._locs[view]

    def __call__(self, a, b):
        la, lb = self.locs(a), self.locs(b)
        m12, _, _ = self.ctx.match_two_sided(a, la, b, lb, self.thr, self.wid)
        src, dst = get_matches(la, lb, m12)
        return src.astype(np.float32), dst.astype(np.float32), len(src)


def StructureFromMotion(imgs, global_set, args, MIN_REPROJECTION_ERROR=0.5, matcher=None,
                        ctx=None, verbose=False):
    """SFM.py:47-88: tracks of consecutive-pair correspondences into global_set.

    matcher(a, b) -> (query float32 (n, 2), train float32 (n, 2), n); default:
    HarrisMatcher on an MvsContext of imgs (ctx, created if not given).  The
    reprojection test and the GlobalSet merge follow the reference; bundle
    adjustment is not run (it moves world points only)."""
    if getattr(args, "nonSeq", False):
        raise NotImplementedError
    par_K, par_r, par_t = read_pars(args)
    K, R, t = pars_to_arrays(par_K, par_r, par_t, len(imgs))
    if matcher is None:
        if ctx is None:
            from .MVS2 import scene_context
            ctx = scene_context(imgs, par_K, par_r, par_t)
        matcher = HarrisMatcher(ctx)
    stats = {"pairs": 0, "correspondences": 0, "kept": 0}
    for a, b in sequence_pairs(len(imgs)):
        q, tr, n = matcher(a, b)
        if verbose:
            print("inliers_n:", n)
        stats["pairs"] += 1
        if n == 0:
            continue
        q = np.ascontiguousarray(q, np.float32).reshape(-1, 2)
        tr = np.ascontiguousarray(tr, np.float32).reshape(-1, 2)
        pts, keep = _lib.sfm_pair(K[a], R[a], t[a], K[b], R[b], t[b], q, tr, MIN_REPROJECTION_ERROR)
        stats["correspondences"] += int(n)
        stats["kept"] += int(keep.sum())
        for k in np.nonzero(keep)[0]:
            global_set.add2pts([(a, q[k][0], q[k][1]), (b, tr[k][0], tr[k][1])], pts[k])
    return stats

"""Drop-in for the reference's MVS stage (MVS2.py), running on MI355X.

DensePointsWithMVS2(imgs, global_set, args)   MVS2.py:176-295
    Same arguments, prints and side effects (initial_patches.ply,
    all_patches.ply in the working directory).  Seeding, the 100k-pop FIFO
    expansion and the cell-table output order run in libmvs_amd.so: photo
    tests on the GPU (HIP, gfx950), the order-dependent commit on the host.
MyPatch.photo_consistenecy_test(...)          MVS2.py:62-77
    Same method on the same fields; one-candidate call of the batched GPU
    scorer.  Use photo_consistency_batch for many candidates.
"""
import sys
import time
import zlib

import numpy as np

from . import _lib
from .utils import export2ply, pars_to_arrays, read_pars, tracks_to_arrays

last_stats = {}
_ctx_cache = {}


def _device_index():
    import os
    return int(os.environ.get("LOCAL_RANK", os.environ.get("MVS_DEVICE", "0")))


def _images_key(imgs):
    """Identity and a content fingerprint of the image list: the element
    arrays' ids, buffers and shapes, and a CRC of every 5th pixel of every
    61st row of each image (~0.15 MB for dinoRing's 48 views, so the
    per-candidate drop-in stays cheap).  The reference re-reads imgs on every
    photo test; a caller that replaces an array, or rewrites sampled pixels in
    place, gets a fresh context.  (A change confined to unsampled pixels is
    not seen: call clear_context_cache().)"""
    parts = [id(imgs), len(imgs)]
    crc = 0
    for a in imgs:
        a = np.asarray(a)
        parts += [id(a), a.shape, a.__array_interface__["data"][0]]
        crc = zlib.crc32(np.ascontiguousarray(a[::61, ::5]).tobytes(), crc)
    parts.append(crc)
    return tuple(parts)


def clear_context_cache():
    """Forget the cached GPU context (e.g. after editing images in place).  The
    context itself is not closed here: whoever still holds it (a running
    Stage, an SfM matcher) keeps a valid handle, and it is destroyed when the
    last reference goes."""
    _ctx_cache.clear()


def scene_context(imgs, par_K, par_r, par_t, device=None):
    """MvsContext for (imgs, cameras), cached on the images (identity + a
    sampled content fingerprint, _images_key) and the camera values (SfM and
    MVS each call read_pars, MVS2.py:178 / SFM.py:54)."""
    K, R, t = pars_to_arrays(par_K, par_r, par_t, len(imgs))
    key = (_images_key(imgs), K.tobytes(), R.tobytes(), t.tobytes())
    ctx = _ctx_cache.get(key)
    if ctx is None:
        ctx = _lib.MvsContext(imgs, K, R, t, device=_device_index() if device is None else device)
        clear_context_cache()
        _ctx_cache[key] = (ctx, imgs)
        return ctx
    return ctx[0]


class MyPatch(object):
    """Patch record with the reference's fields (MVS2.py:45-57)."""

    def __init__(self, centroid, normal, reference_img_index, visible_set, color, dist, patch_size=5):
        self.dist = dist
        self.c = centroid
        self.n = normal
        self.R = reference_img_index
        self.V = visible_set if visible_set is not None else []
        self.color = color
        self.patch_size = patch_size
        self.avg_ncc_score = 0

    def visible_ct(self):
        return len(self.V)

    def photo_consistenecy_test(self, imgs, par_K, par_r, par_t, MIN_NCC=0.7):
        ctx = scene_context(imgs, par_K, par_r, par_t)
        xy, mask, count, avg = ctx.score(np.asarray(self.c, np.float64)[None], [self.R], MIN_NCC, 5)
        for idx in _mask_views(mask[0]):
            self.V.append([idx, xy[0, 0], xy[0, 1]])
        # the reference's own sum of the passing nccs / |V| (MVS2.py:73-76), bit-exact
        self.avg_ncc_score = float(ctx.exact_avg([self.R], xy, mask, 5)[0]) if count[0] else 0
        return self.V


def _mask_views(words):
    out = []
    for w, m in enumerate(np.asarray(words, np.uint64)):
        m = int(m)
        while m:
            b = (m & -m).bit_length() - 1
            out.append(64 * w + b)
            m &= m - 1
    return out


def photo_consistency_batch(ctx, centroids, ref_views, MIN_NCC=0.7, wid=5):
    """Batched photo test: (xy, mask, count, avg) per candidate."""
    return ctx.score(centroids, ref_views, MIN_NCC, wid)


def DensePointsWithMVS2(imgs, global_set, args, max_pops=100000, device=None):
    """MVS2.py:176-295 on the GPU.  Returns None like the reference; the run's
    counters are left in MVS2.last_stats.

    Under torch.distributed with world size > 1 (one process per GPU), the
    expansion sweeps are sharded across ranks (parallel.stage_sharded); every
    rank ends with the same patches and rank 0 writes the PLY files.

    `args.filter_outliers` (opt-in, default off) runs CellTable.filter_out_outlier
    (MVS2.py:132-158) before the reconstruction, as if the reference's
    commented-out call at MVS2.py:281 were enabled, with its prints."""
    t0 = time.time()
    filter_outliers = bool(getattr(args, "filter_outliers", False))
    par_K, par_r, par_t = read_pars(args)
    n_observations, n_world_points, legal_sets = global_set.getInfo()
    track_off, obs_view, obs_xy = tracks_to_arrays(legal_sets)
    ctx = scene_context(imgs, par_K, par_r, par_t, device)
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    if world > 1:
        from . import parallel
        initial, allp, stats = parallel.stage_sharded(
            ctx, track_off, obs_view, obs_xy, cell_size=args.cell_size, scale=args.scale, wid=5,
            max_pops=max_pops, device=device, filter_outliers=filter_outliers)
        if dist.get_rank() != 0:
            last_stats.clear()
            last_stats.update(stats)
            return None
    else:
        initial, allp, stats = ctx.stage(track_off, obs_view, obs_xy, cell_size=args.cell_size,
                                         scale=args.scale, wid=5, max_pops=max_pops,
                                         filter_outliers=filter_outliers)
    print("len of initial patches", len(initial))
    export2ply(initial[:, :3], initial[:, 3:], path="initial_patches")
    print("filter outliers")
    if filter_outliers:
        # filter_out_outlier's own prints (MVS2.py:155), one per removed Q-table entry
        left = stats["outlier_lines"]
        while left > 0:
            k = min(left, 1 << 16)
            sys.stdout.write("remove a outlier\n" * k)
            left -= k
    print("reconstruct point cloud")
    t1 = time.time()
    print("Optimization took {0:.0f} seconds".format(t1 - t0))
    print("points len:", len(allp))
    export2ply(allp[:, :3], allp[:, 3:], path="all_patches")
    stats["seconds"] = t1 - t0
    last_stats.clear()
    last_stats.update(stats)
    return None

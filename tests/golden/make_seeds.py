"""Synthetic SfM seed tracks for dinoRing (test infrastructure).

The reference's SfM stage (ORB + FLANN + RANSAC, utils.py:160-232) needs
OpenCV, which the image lacks, so the MVS stage's input -- GlobalSet tracks
whose point2d_list is [(view, x: float32, y: float32), ...] (GlobalSet.py:36-50,
consumed at MVS2.py:208-250) -- is manufactured here:

  for consecutive views (a, a+1): textured pixels (gray > 60, |grad| > 8) inside
  rows [20, 460) x cols [20, 620), shuffled with default_rng(0); sweep 400
  depths z in [0.58, 0.74] m along the pixel's ray; keep the best 11x11 NCC in
  view a+1 (window at the rounded projection) if > 0.95; at most 30 per pair.
  Every coordinate is jittered by U(-0.25, 0.25) (default_rng(1)) and cast to
  float32: exactly epipolar-consistent seeds sit on integer-truncation knife
  edges.
"""
import glob
import os

import numpy as np


def read_par(path):
    """Middlebury *_par.txt (same parse as utils.read_pars, utils.py:56-81)."""
    K, R, t = [], [], []
    with open(path) as f:
        lines = f.readlines()
    for line in lines[1:]:
        tp = [float(v) for v in line.split()[1:]]
        K.append(np.array(tp[0:9]).reshape(3, 3))
        R.append(np.array(tp[9:18]).reshape(3, 3))
        t.append(np.array(tp[18:21]).reshape(3, 1))
    return np.array(K), np.array(R), np.array(t)


def load_dino(data_dir):
    from PIL import Image
    files = sorted(glob.glob(os.path.join(data_dir, "*.png")))
    imgs = [np.asarray(Image.open(f).convert("RGB")).copy() for f in files]
    K, R, t = read_par(glob.glob(os.path.join(data_dir, "*_par.txt"))[0])
    return imgs, K, R, t


def _gray(img):
    p = img.astype(np.int64)
    return ((p[..., 0] * 1868 + p[..., 1] * 9617 + p[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)


def _ncc_rows(a, B):
    a = a.astype(np.float64) - a.mean()
    B = B.astype(np.float64) - B.mean(1, keepdims=True)
    den = np.sqrt((a * a).sum() * (B * B).sum(1))
    with np.errstate(all="ignore"):
        return np.where(den > 0, (B @ a) / den, -1.0)


def make_seeds(imgs, K, R, t, per_pair=30, max_try=1500, wid=5):
    V = len(imgs)
    H, W = imgs[0].shape[:2]
    gray = [_gray(im) for im in imgs]
    rng0 = np.random.default_rng(0)
    zs = np.linspace(0.58, 0.74, 400)
    off, obs_v, obs_xy = [0], [], []
    for a in range(V - 1):
        b = a + 1
        g = gray[a].astype(np.float64)
        gy, gx = np.gradient(g)
        m = (g > 60) & (np.hypot(gx, gy) > 8)
        m[:20] = False; m[460:] = False; m[:, :20] = False; m[:, 620:] = False
        ys, xs = np.nonzero(m)
        order = rng0.permutation(len(ys))
        Kinv = np.linalg.inv(K[a])
        found = 0
        for idx in order[:max_try]:
            y, x = int(ys[idx]), int(xs[idx])
            ray = Kinv @ np.array([x, y, 1.0])
            Xw = (zs[:, None] * ray[None, :] - t[a].ravel()[None, :]) @ R[a]     # R^T (z ray - t)
            p = (Xw @ R[b].T + t[b].ravel()[None, :]) @ K[b].T
            u, v = p[:, 0] / p[:, 2], p[:, 1] / p[:, 2]
            ui, vi = np.rint(u).astype(int), np.rint(v).astype(int)
            ok = (vi - wid >= 0) & (vi + wid + 1 < H) & (ui - wid > 0) & (ui + wid + 1 < W)
            if not ok.any():
                continue
            wa = gray[a][y - wid:y + wid + 1, x - wid:x + wid + 1].ravel()
            cand = np.nonzero(ok)[0]
            Bw = np.stack([gray[b][vi[k] - wid:vi[k] + wid + 1, ui[k] - wid:ui[k] + wid + 1].ravel()
                           for k in cand])
            s = _ncc_rows(wa, Bw)
            k = int(np.argmax(s))
            if s[k] > 0.95:
                j = cand[k]
                obs_v += [a, b]
                obs_xy += [[x, y], [u[j], v[j]]]
                off.append(len(obs_v))
                found += 1
                if found >= per_pair:
                    break
    obs_xy = np.array(obs_xy, np.float64)
    obs_xy += np.random.default_rng(1).uniform(-0.25, 0.25, obs_xy.shape)
    return {"track_off": np.array(off, np.int64), "obs_view": np.array(obs_v, np.int32),
            "obs_xy": obs_xy.astype(np.float32)}


def subset_seeds(seeds, n_views):
    """The tracks whose every observation lies in views 0..n_views-1 (the
    47-view dinoRing subset standing in for BASELINE config 3's 47 views;
    templeRing itself is absent)."""
    off, ov, oxy = seeds["track_off"], seeds["obs_view"], seeds["obs_xy"]
    keep_off, keep_v, keep_xy = [0], [], []
    for k in range(len(off) - 1):
        v = ov[off[k]:off[k + 1]]
        if (v < n_views).all():
            keep_v += list(v)
            keep_xy += list(oxy[off[k]:off[k + 1]])
            keep_off.append(len(keep_v))
    return (np.array(keep_off, np.int64), np.array(keep_v, np.int32),
            np.array(keep_xy, np.float32).reshape(-1, 2))

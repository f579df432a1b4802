"""Synthetic workloads of SURVEY.md section 8(d) (bench and tests).

candidates(): config 2/4 candidate batch -- reference view R ~ U{0..V-1},
  pixel (x, y) ~ U{6..W-7} x U{5..H-8} + U[0,1) sub-pixel, centre = back-projection
  of (x, y) through camera R at depth z ~ U(0.60, 0.72) m.
ring_scene(): config 4 -- V views of uniform-random RGB textures on a ring of
  radius 0.66 m looking at the origin, K = dinoRing's scaled to W x H.
"""
import numpy as np


def candidates(n, K, R, t, W=640, H=480, seed=0):
    V = len(K)
    K = np.asarray(K, np.float64).reshape(V, 3, 3)
    R = np.asarray(R, np.float64).reshape(V, 3, 3)
    t = np.asarray(t, np.float64).reshape(V, 3)
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, V, n).astype(np.int32)
    x = rng.integers(6, W - 6, n) + rng.random(n)
    y = rng.integers(5, H - 7, n) + rng.random(n)
    z = rng.uniform(0.60, 0.72, n)
    Kinv = np.linalg.inv(K)
    ray = np.einsum("nij,nj->ni", Kinv[ref], np.stack([x, y, np.ones(n)], 1))
    cam = z[:, None] * ray - t[ref]
    c = np.einsum("nji,nj->ni", R[ref], cam)
    return np.ascontiguousarray(c), ref


def ring_scene(V=256, H=1080, W=1920, seed=0, radius=0.66):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (V, H, W, 3), dtype=np.uint8)
    f = 3310.4 * W / 640.0
    K = np.tile(np.array([[f, 0, W / 2], [0, f, H / 2], [0, 0, 1.0]]), (V, 1, 1))
    R = np.empty((V, 3, 3))
    t = np.empty((V, 3))
    for v in range(V):
        a = 2 * np.pi * v / V
        C = np.array([radius * np.cos(a), radius * np.sin(a), 0.05 * np.sin(3 * a)])
        z = -C / np.linalg.norm(C)
        up = np.array([0, 0, 1.0])
        x = np.cross(up, z); x /= np.linalg.norm(x)
        y = np.cross(z, x)
        R[v] = np.stack([x, y, z])
        t[v] = -R[v] @ C
    return rgb, K, R, t

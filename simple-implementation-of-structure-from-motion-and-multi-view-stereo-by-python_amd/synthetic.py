"""Synthetic workloads of SURVEY.md section 8(d) (bench and tests).

candidates(): config 2/4 candidate batch -- reference view R ~ U{0..V-1},
  pixel (x, y) ~ U{6..W-7} x U{5..H-8} + U[0,1) sub-pixel, centre = back-projection
  of (x, y) through camera R at depth z ~ U(0.60, 0.72) m.
ring_scene(): config 4 -- V views of uniform-random RGB textures on a ring of
  radius 0.66 m looking at the origin, K = dinoRing's scaled to W x H.
sphere_scene(): a geometrically consistent scene for stage tests -- a
  procedurally textured sphere at the origin rendered into ring cameras
  (black background), plus 2-view seed tracks on its surface.
sphere_scene_device(): the same kind of scene at config-4 size (256 views of
  1920x1080), rendered on the GPU with torch (test/bench data generation only),
  so that sweeps over it accept candidates.
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


def ring_cameras(V, H, W, radius=0.66):
    f = 3310.4 * W / 640.0
    K = np.tile(np.array([[f, 0, W / 2], [0, f, H / 2], [0, 0, 1.0]]), (V, 1, 1))
    R = np.empty((V, 3, 3))
    t = np.empty((V, 3))
    for v in range(V):
        a = 2 * np.pi * v / V
        C = np.array([radius * np.cos(a), radius * np.sin(a), 0.05 * np.sin(3 * a)])
        z = -C / np.linalg.norm(C)
        up = np.array([0, 0, 1.0])
        x = np.cross(up, z)
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        R[v] = np.stack([x, y, z])
        t[v] = -R[v] @ C
    return K, R, t


def ring_scene(V=256, H=1080, W=1920, seed=0, radius=0.66):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (V, H, W, 3), dtype=np.uint8)
    K, R, t = ring_cameras(V, H, W, radius)
    return rgb, K, R, t


def _first_hit(O, d, rad):
    """Ray parameter of the first intersection with |X| = rad (nan if none)."""
    b = d @ O if d.ndim == 1 else np.einsum("...i,i->...", d, O)
    disc = b * b - (O @ O - rad * rad)
    s = -b - np.sqrt(np.where(disc > 0, disc, np.nan))
    return np.where(s > 0, s, np.nan)


def sphere_scene(V=24, H=96, W=128, seed=0, rad=0.02, n_seeds=300, camera_radius=0.33):
    """Images of a textured sphere seen by V ring cameras, and 2-view seed
    tracks (track_off, obs_view, obs_xy float32) of sphere points seen in
    views a and a+1, coordinates jittered by U(-0.25, 0.25) px."""
    rng = np.random.default_rng(seed)
    K, R, t = ring_cameras(V, H, W, camera_radius)
    freqs = rng.normal(0, 1, (6, 3)) * 18.0
    phases = rng.uniform(0, 2 * np.pi, 6)

    def tex(X):
        nrm = X / rad
        return np.clip(128 + 20 * sum(np.sin(nrm @ f + p) for f, p in zip(freqs, phases)), 0, 255)

    rgb = np.zeros((V, H, W, 3), np.uint8)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    pix = np.stack([xs + 0.5, ys + 0.5, np.ones_like(xs)], -1)
    for v in range(V):
        d = pix @ np.linalg.inv(K[v]).T @ R[v]
        d /= np.linalg.norm(d, axis=-1, keepdims=True)
        O = -R[v].T @ t[v]
        s = _first_hit(O, d, rad)
        hit = np.isfinite(s)
        X = O + np.where(hit, s, 0.0)[..., None] * d
        g = np.where(hit, tex(X), 0.0)
        rgb[v] = np.stack([g, 0.9 * g, 0.8 * g], -1).astype(np.uint8)
    off, ov, oxy = [0], [], []
    for _ in range(n_seeds):
        a = int(rng.integers(0, V))
        b = (a + 1) % V
        for _try in range(50):
            x, y = rng.uniform(8, W - 8), rng.uniform(8, H - 8)
            d = R[a].T @ (np.linalg.inv(K[a]) @ np.array([x, y, 1.0]))
            d /= np.linalg.norm(d)
            O = -R[a].T @ t[a]
            s = _first_hit(O, d, rad)
            if not np.isfinite(s):
                continue
            P = O + s * d
            pb = K[b] @ (R[b] @ P + t[b])
            u, w = pb[0] / pb[2], pb[1] / pb[2]
            if not (8 < u < W - 8 and 8 < w < H - 8):
                continue
            j = rng.uniform(-0.25, 0.25, 4)
            ov += [a, b]
            oxy += [(x + j[0], y + j[1]), (u + j[2], w + j[3])]
            off.append(len(ov))
            break
    return (rgb, K, R, t, np.array(off, np.int64), np.array(ov, np.int32),
            np.array(oxy, np.float32).reshape(-1, 2))


def sphere_scene_device(V=256, H=1080, W=1920, rad=0.03, camera_radius=0.66, seed=0, device="cuda"):
    """A textured sphere of radius `rad` at the origin seen by V ring cameras
    (ring_cameras: dinoRing's K scaled to W x H), black background; rendered
    per view on `device` with torch.  Returns host (rgb (V,H,W,3) uint8, K, R, t).
    The texture is a sum of six sinusoids of the surface direction with
    periods of a few hundred pixels at this size, so neighbouring views agree
    at the same pixel (the photo test compares every view at the reference
    view's pixel, MVS2.py:68) and sweeps accept candidates."""
    import torch
    rng = np.random.default_rng(seed)
    K, R, t = ring_cameras(V, H, W, camera_radius)
    freqs = torch.tensor(rng.normal(0, 1, (6, 3)) * 6.0, dtype=torch.float64, device=device)
    phases = torch.tensor(rng.uniform(0, 2 * np.pi, 6), dtype=torch.float64, device=device)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float64, device=device),
                            torch.arange(W, dtype=torch.float64, device=device), indexing="ij")
    pix = torch.stack([xs + 0.5, ys + 0.5, torch.ones_like(xs)], -1)
    out = np.empty((V, H, W, 3), np.uint8)
    for v in range(V):
        Kinv = torch.tensor(np.linalg.inv(K[v]), device=device)
        Rv = torch.tensor(R[v], device=device)
        d = pix @ Kinv.T @ Rv
        d = d / d.norm(dim=-1, keepdim=True)
        O = torch.tensor(-R[v].T @ t[v], device=device)
        b = d @ O
        disc = b * b - (O @ O - rad * rad)
        hit = disc > 0
        s = -b - torch.sqrt(torch.clamp(disc, min=0))
        X = O + s.unsqueeze(-1) * d
        nrm = X / rad
        g = 128 + 20 * torch.sin(nrm @ freqs.T + phases).sum(-1)
        g = torch.where(hit, torch.clamp(g, 0, 255), torch.zeros_like(g))
        rgb = torch.stack([g, 0.9 * g, 0.8 * g], -1).to(torch.uint8)
        out[v] = rgb.cpu().numpy()
    return out, K, R, t

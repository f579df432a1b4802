"""GPU debug: tiled scorer vs oracle on the bench distribution; prints the
mismatching candidates with the binary32 decision quantities of each view
(usage: python tools/debug_mma.py WID THR [N])."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests")]
os.environ["MVS_SCORE_KERNEL"] = "tiled"
import importlib  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from make_seeds import load_dino  # noqa: E402
from conftest import bench_candidates  # noqa: E402

wid, thr = int(sys.argv[1]), float(sys.argv[2])
N = int(sys.argv[3]) if len(sys.argv) > 3 else 6000
pkg = importlib.import_module("simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd")
imgs, K, R, t = load_dino(os.path.join(REPO, "data", "dinoRing"))
rgb = np.stack(imgs)
sc = orc.Scene(rgb, K, R, t)
gray = np.stack([orc.gray_from_rgb(x) for x in rgb]).astype(np.int64)
V, H, W = gray.shape
c, ref = bench_candidates(N, K, R, t, seed=wid)
with pkg.MvsContext(rgb, K, R, t, device=0) as ctx:
    xy, mask, count, avg = ctx.score(c, ref, thr, wid)
    hits = ctx.exact_hits() if hasattr(ctx, "exact_hits") else None
oxy, omask, ocount, oavg = sc.score_batch(c, ref, thr, wid, nthreads=8)
bad = np.nonzero((mask != omask).any(1) | (count != ocount))[0]
print("mismatches", len(bad), "of", N, "exact_hits", hits)
n = (2 * wid + 1) ** 2
for k in bad[:10]:
    x, y = oxy[k]
    q, r = int(x), int(y)
    Rk = ref[k]
    win = gray[:, r - wid:r + wid + 1, q - wid:q + wid + 1].reshape(V, -1) - 128
    S = win.sum(1); Q = (win * win).sum(1)
    db = n * Q - S * S
    w = np.where(db > 0, 1 / np.sqrt(np.maximum(db, 1).astype(np.float64)), np.nan)
    num = n * (win @ win[Rk]) - S[Rk] * S
    T = np.float32(thr * (n - 1) / n / w[Rk])
    xx = (np.float32(num) * np.float32(w) - T).astype(np.float32)
    diff = int(mask[k, 0]) ^ int(omask[k, 0])
    print(f"cand {k} R {Rk} px ({q},{r}) tile ({q // 16},{r // 8}) rel ({q % 16},{r % 8}) gpu cnt {count[k]} "
          f"oracle {ocount[k]} diff views {[v for v in range(V) if diff >> v & 1]}")
    for v in [v for v in range(V) if diff >> v & 1][:4]:
        print(f"   v {v}: num {num[v]} w {w[v]:.6g} T {T:.6g} x {xx[v]:.6g} gpu {int(mask[k,0]) >> v & 1} "
              f"oracle {int(omask[k,0]) >> v & 1} S_b {S[v]} db {db[v]}")

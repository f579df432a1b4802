import sys, os, importlib, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests/golden')
from make_seeds import load_dino
from oracle import oracle as orc
pkg = importlib.import_module("simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd")
imgs, K, R, t = load_dino('/root/repo/data/dinoRing')
rgb = np.stack(imgs)
sc = orc.Scene(rgb, K, R, t)
ctx = pkg.MvsContext(rgb, K, R, t)
rng = np.random.default_rng(0)
# parents: on-surface candidates from the bench distribution that pass the photo test
c, ref = pkg.synthetic.candidates(20000, K, R, t, seed=3)
xy, mask, count, avg = ctx.score(c, ref, 0.4, 5)
sel = np.nonzero(count >= 3)[0][:300]
O = np.array([-(R[v].T @ t[v].ravel()) for v in range(48)])
pc = c[sel]; pxy = xy[sel]
pn = (O[ref[sel]] - pc); pn /= np.linalg.norm(pn, axis=1)[:, None]
jp, jv, jd = [], [], []
for k, i in enumerate(sel):
    m = int(mask[i, 0])
    for v in range(48):
        if m >> v & 1:
            for d in (-1, 1):
                jp.append(k); jv.append(v); jd.append(d)
g = ctx.expand_candidates(pc, pn, pxy, jp, jv, jd)
o = sc.expand_candidates(pc, pn, pxy, jp, jv, jd)
names = ['X', 'nX', 'color', 'xy', 'mask', 'count', 'accept']
for nm, a, b in zip(names, g, o):
    eq = np.array_equal(a, b)
    print(nm, eq, '' if eq else (np.nonzero((a != b).reshape(len(a), -1).any(1))[0][:10], a[(a != b).reshape(len(a), -1).any(1)][:3], b[(a != b).reshape(len(a), -1).any(1)][:3]))
print('jobs', len(jp), 'accepted', int(g[6].sum()), int(o[6].sum()))

import importlib, sys
import numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests/golden')
from make_seeds import load_dino
pkg = importlib.import_module("simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd")
imgs, K, R, t = load_dino('/root/repo/data/dinoRing'); rgb = np.stack(imgs)
s = dict(np.load('/root/repo/tests/golden/seeds_dino.npz'))
args = (s["track_off"], s["obs_view"], s["obs_xy"])
ref_ctx = pkg.MvsContext(rgb, K, R, t)
ini, allp, st = ref_ctx.stage(*args, cell_size=2, scale=10.0, wid=5, max_pops=100000)
ini2, allp2, st2 = ref_ctx.stage(*args, cell_size=2, scale=10.0, wid=5, max_pops=100000)
print("single-run repeat equal:", np.array_equal(allp, allp2), st == st2)
for world in (1, 2, 3):
    ctxs = [pkg.MvsContext(rgb, K, R, t) for _ in range(world)]
    sts = [c.stage_begin(*args, cell_size=2, scale=10.0, wid=5, max_pops=100000, rank=r, world=world) for r, c in enumerate(ctxs)]
    dev = torch.device("cuda", 0)
    while True:
        njs = [x.plan() for x in sts]
        if njs[0] == 0: break
        smax = sts[0].slice_max(njs[0])
        outs = [torch.full((smax, sts[0].width), -7, dtype=torch.int64, device=dev) for _ in range(world)]
        if world == 1:
            sts[0].score_slice(None); sts[0].ingest(None); continue
        for x, o in zip(sts, outs): x.score_slice(o)
        allbuf = torch.stack(outs)
        for x in sts: x.ingest(allbuf)
    res = [x.finish() for x in sts]
    for r, (a, b, c) in enumerate(res):
        d = (b != allp).any(1) if b.shape == allp.shape else None
        print(f"world {world} rank {r}: rows {len(b)} equal {np.array_equal(b, allp)} ini {np.array_equal(a, ini)}",
              "" if d is None else f"diff rows {int(d.sum())} first {int(np.argmax(d))}", c == st)
    for x in sts: x.close()
    for c in ctxs: c.close()

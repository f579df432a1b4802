"""Randomised parity sweep of k_score_tab's band queues (one per XCD) and
the two counter sets: dense batches (implicit items, >= 64 candidates per
tile) and sparse ones (k_item_scan) on small scenes of odd sizes, with the
scorer's grid held to several sizes (mvs_set_scorer_grid: bands with
unequal workgroup counts, bands smaller than their static items), on two
streams in turn -- every output against the oracle.  Exit 1 on a mismatch."""
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, '/root/repo')
pkg = importlib.import_module("simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd")
from oracle import oracle as orc  # noqa: E402

syn = pkg.synthetic
rng = np.random.default_rng(11)
dev = torch.device("cuda:0")
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
bad = cases = 0
for V in (8, 20, 48, 64):
    H = int(rng.integers(60, 140)); W = int(rng.integers(70, 210))
    rgb, K, R, t = syn.ring_scene(V=V, H=H, W=W, seed=V + 2000)
    rgb = ((rgb.astype(np.uint16) + np.roll(rgb, 1, axis=0) + np.roll(rgb, 1, axis=1)) // 3).astype(np.uint8)
    sc = orc.Scene(rgb, K, R, t)
    ntiles = ((W + 15) // 16) * ((H + 7) // 8)
    with pkg.MvsContext(rgb, K, R, t, device=0) as cx:
        for dense in (True, False):
            n = 96 * ntiles if dense else max(2048, 8 * ntiles)
            c, ref = syn.candidates(n, K, R, t, W=W, H=H, seed=V + n)
            exp = sc.score_batch(c, ref, 0.7, 5, nthreads=16)
            tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
            for k, grid in enumerate((0, 37, 8, 100, 333)):
                cases += 1
                xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
                rec = torch.full((n, 2), -1, dtype=torch.int64, device=dev)
                s = streams[k % 2]
                torch.cuda.synchronize()
                cx.set_scorer_grid(grid)
                cx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=s.cuda_stream)
                s.synchronize()
                cx.set_scorer_grid(0)
                r = rec.cpu().numpy()
                m = r[:, 0].view(np.uint64)
                ok = (np.array_equal(xy.cpu().numpy(), exp[0]) and np.array_equal(m, exp[1][:, 0])
                      and np.array_equal(np.bitwise_count(m).astype(np.int32), exp[2])
                      and np.allclose(r[:, 1].view(np.float64), exp[3], rtol=0, atol=1e-12))
                print(f"V={V} {H}x{W} tiles={ntiles} n={n} {'dense' if dense else 'sparse'} grid={grid}: "
                      f"{'ok' if ok else 'MISMATCH'}", flush=True)
                bad += 0 if ok else 1
print(f"{cases} cases, {bad} mismatches")
sys.exit(1 if bad else 0)

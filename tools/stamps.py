"""Phase cycles of k_score_mma from the -DMVS_STAMPS diagnostic build
(build_lib.py --stamps): per work item, staging (+ the barrier), moments,
candidates (to the item's end barrier), wave 0's own candidate time."""
import ctypes
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["MVS_LIB"] = os.path.join(REPO, "simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd",
                                     "libmvs_amd_stamps.so")
import bench  # noqa: E402

wid = int(sys.argv[1]) if len(sys.argv) > 1 else 5
pkg = importlib.import_module(bench.PKG_NAME)
rgb, K, R, t = bench.load_scene()
n = 1 << 20
c, ref = pkg.synthetic.candidates(n, K, R, t, seed=0)
ctx = pkg.MvsContext(rgb, K, R, t)
lib = pkg._lib.load()
lib.mvs_read_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 8, np.uint64)
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps(buf.ctypes.data)
before = buf.copy()
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps(buf.ctypes.data)
d = (buf - before).reshape(4096, 8).astype(np.float64)
items = d[:, 0]
act = items > 0
tot = items.sum()
print(f"wid {wid}: workgroups with items {act.sum()}, items {tot:.0f}")
for k, name in [(1, "staging"), (2, "moments"), (6, "  hsum"), (7, "  vsum"), (3, "candidates")]:
    print(f"  {name:10s} {d[act, k].sum() / tot:9.0f} cycles per item")
print(f"  wave 0: {d[act, 4].sum() / tot:9.0f} cycles of own candidate work per item, "
      f"{d[act, 5].sum() / tot:.2f} M-blocks per item -> {d[act, 4].sum() / max(d[act, 5].sum(), 1):.0f} cycles per M-block")
per_wg = d[act, 1] + d[act, 2] + d[act, 3]
print(f"  per workgroup {per_wg.mean():.0f} cycles (max {per_wg.max():.0f})")

"""Phase cycles of k_score_mma from the -DMVS_STAMPS diagnostic build
(build_lib.py --stamps): per work item, staging (+ the barrier), moments,
candidates (to the item's end barrier), wave 0's own candidate time."""
import ctypes
import importlib
import os
import sys

import numpy as np

import faulthandler
faulthandler.dump_traceback_later(150, exit=True)   # a stuck run names its line

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["MVS_LIB"] = os.environ.get("STAMPS_LIB") or os.path.join(
    REPO, "simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd", "libmvs_amd_stamps.so")
print("library", os.path.basename(os.environ["MVS_LIB"]))
import bench  # noqa: E402

wid = int(sys.argv[1]) if len(sys.argv) > 1 else 5
scene = sys.argv[2] if len(sys.argv) > 2 else "dino"
pkg = importlib.import_module(bench.PKG_NAME)
n = 1 << 20
if scene == "ring256":   # k_score_mma_v: slot 0 counts (item, view group) units; 6 = phase 3 alone
    import torch
    rgb, K, R, t = pkg.synthetic.sphere_scene_device(256, 1080, 1920, seed=0, device=torch.device("cuda", 0))
    c, ref = pkg.synthetic.candidates(n, K, R, t, W=1920, H=1080, seed=0)
else:
    rgb, K, R, t = bench.load_scene()
    c, ref = pkg.synthetic.candidates(n, K, R, t, seed=0)
print("scene ready", flush=True)
ctx = pkg.MvsContext(rgb, K, R, t)
print("context ready", flush=True)
lib = pkg._lib.load()
lib.mvs_read_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 16, np.uint64)
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps(buf.ctypes.data)
before = buf.copy()
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps(buf.ctypes.data)
d = (buf - before).reshape(4096, 16)[:2048].astype(np.float64)   # rows 2048+: k_bin
items = d[:, 0]
act = items > 0
tot = items.sum()
print(f"wid {wid}: workgroups with items {act.sum()}, items {tot:.0f}")
labels = ([(1, "D table (+ item constants)"), (4, "  wave 0 own D-table work"), (5, "  barrier after phase 2"),
           (6, "  item constants (group 0)"), (2, "MFMA tasks"), (7, "  wave 0 prefetch + own task"),
           (3, "next region lands + phase 4")]
          if scene == "ring256" else
          [(1, "staging"), (2, "moments"), (6, "  hsum"), (7, "  vsum"), (3, "candidates")])
for k, name in labels:
    print(f"  {name:28s} {d[act, k].sum() / tot:9.0f} cycles per {'(item, group)' if scene == 'ring256' else 'item'}")
if scene == "ring256":
    g0 = tot / 4.0
    print(f"  group-0 barrier after phase 2 {d[act, 8].sum() / g0:9.0f} cycles per group 0; other groups "
          f"{(d[act, 5].sum() - d[act, 8].sum()) / max(tot - g0, 1):9.0f}")
    print(f"  phase-2 own work, mean of the 16 waves {d[act, 9].sum() / tot / 16:9.0f}; wave 0 prefetch + stores "
          f"{d[act, 10].sum() / tot:9.0f}")
    print(f"  phase-3 tasks {d[act, 12].sum() / tot:.2f} per (item, group), {d[act, 11].sum() / max(d[act, 12].sum(), 1):9.0f} cycles each")
if scene != "ring256":
  print(f"  wave 0: {d[act, 4].sum() / tot:9.0f} cycles of own candidate work per item, "
      f"{d[act, 5].sum() / tot:.2f} M-blocks per item -> {d[act, 4].sum() / max(d[act, 5].sum(), 1):.0f} cycles per M-block")
if scene != "ring256" and d[act, 13].sum() > 0:
    print(f"  wave 0 final-barrier wait {d[act, 8].sum() / tot:9.0f} cycles per item; own phase-3 time: "
          f"slowest wave {d[act, 9].sum() / tot:9.0f}, mean of the 16 waves {d[act, 10].sum() / tot / 16:9.0f}")
    print(f"  units {d[act, 13].sum() / tot:.2f} per item, {d[act, 12].sum() / max(d[act, 13].sum(), 1) * 100:.1f} % span > KSK; "
          f"fix-list appends {d[act, 11].sum() / tot:.2f} per item")
kb = (buf - before).reshape(4096, 16)[2048:].astype(np.float64)
kact = kb[:, 0] > 0
if kact.any():
    print(f"  k_bin: {kact.sum()} workgroups; per workgroup: projection + LDS ranks {kb[kact, 1].mean():.0f}, "
          f"global tile bases {kb[kact, 2].mean():.0f}, bucket writes + ticket {kb[kact, 3].mean():.0f} cycles; "
          f"item scan (last workgroup) {kb[kact, 4].sum():.0f} cycles")
per_wg = d[act, 1] + d[act, 2] + d[act, 3]
print(f"  per workgroup {per_wg.mean():.0f} cycles (max {per_wg.max():.0f})")

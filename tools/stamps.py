"""Phase times of the tiled kernel from the -DMVS_STAMPS diagnostic build."""
import ctypes, importlib, os, sys
import numpy as np
import torch
sys.path.insert(0, '/root/repo')
os.environ["MVS_LIB"] = "/root/repo/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd_stamps.so"
import bench
pkg = importlib.import_module(bench.PKG_NAME)
rgb, K, R, t = bench.load_scene()
n = 1 << 20
c, ref = pkg.synthetic.candidates(n, K, R, t, seed=0)
ctx = pkg.MvsContext(rgb, K, R, t)   # MVS_VARIANT picks the kernel
lib = pkg._lib.load()
lib.mvs_read_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 8, np.uint64)
ctx.score(c, ref, 0.7, 5)            # warm (moments built)
lib.mvs_read_stamps(buf.ctypes.data)
before = buf.copy()
ctx.score(c, ref, 0.7, 5)
lib.mvs_read_stamps(buf.ctypes.data)
d = (buf - before).reshape(4096, 8).astype(np.float64)
items = d[:, 0]
act = items > 0
print("workgroups with items:", act.sum(), "items:", items.sum())
for k, name in [(1, "stage"), (2, "candidates"), (3, "write-out")]:
    print(f"{name:12s} mean per item {d[act, k].sum() / items.sum():10.0f} cycles   total per wg {d[act, k].mean():12.0f}")
if d[:, 4].sum() > 0:
    print(f"wave0 mfma rows  {d[act, 4].sum() / items.sum():10.0f} cycles per item; "
          f"epilogue {d[act, 5].sum() / items.sum():10.0f}; wave0 candidates per item {d[act, 6].sum() / items.sum():.1f}")
print("per-wg total", (d[act, 1] + d[act, 2] + d[act, 3]).mean(), "cycles; max", (d[act, 1] + d[act, 2] + d[act, 3]).max())

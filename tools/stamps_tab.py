"""Phase cycles of k_score_tab from the -DMVS_STAMPS diagnostic build
(build_lib.py --stamps): per item and per wave, the barrier wait at the
round's start, the wave's row-pair sort, its units (K-loops, epilogues)."""
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
pkg = importlib.import_module(bench.PKG_NAME)
n = 1 << 20
rgb, K, R, t = bench.load_scene()
c, ref = pkg.synthetic.candidates(n, K, R, t, seed=0)
ctx = pkg.MvsContext(rgb, K, R, t)
lib = pkg._lib.load()
lib.mvs_read_stamps_tab.argtypes = [ctypes.c_void_p]
buf = np.zeros(1024 * 16, np.uint64)
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps_tab(buf.ctypes.data)
before = buf.copy()
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps_tab(buf.ctypes.data)
d = (buf - before).reshape(1024, 16)[:512].astype(np.float64)
items = d[:, 0].sum()
waves = items * 8
print(f"wid {wid}: items {items:.0f} over {(d[:, 0] > 0).sum()} workgroups; M-blocks {d[:, 4].sum():.0f}")
for k, name in [(1, "barrier wait (round start)"), (2, "DMA issue + sort"), (7, "  DMA issue + loads"), (3, "units"),
                (5, "  K-loops"), (6, "  epilogues")]:
    print(f"  {name:28s} {d[:, k].sum() / waves:9.0f} cycles per (item, wave)")
print(f"  per M-block: K-loop {d[:, 5].sum() / d[:, 4].sum():.0f}, epilogue {d[:, 6].sum() / d[:, 4].sum():.0f} cycles")
# workgroup start / end (100 MHz clock, slots 10 and 11): the kernel's start-up and tail
raw = (buf - before).reshape(1024, 16)[:512]
st, en = raw[:, 10].astype(np.int64), raw[:, 11].astype(np.int64)
ok = (st > 0) & (en > 0)
if ok.any():
    t0 = st[ok].min()
    s_us, e_us = (st[ok] - t0) / 100.0, (en[ok] - t0) / 100.0
    q = lambda a, p: float(np.percentile(a, p))
    print(f"  workgroup start (us after the first): median {q(s_us, 50):.1f}, max {s_us.max():.1f}")
    print(f"  workgroup end: min {e_us.min():.1f}, 10% {q(e_us, 10):.1f}, median {q(e_us, 50):.1f}, "
          f"90% {q(e_us, 90):.1f}, max {e_us.max():.1f} us")
    hw = raw[:, 12].astype(np.int64)[ok] - 1
    xcc = (raw[:, 13].astype(np.int64)[ok] - 1) & 15
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    per_item = e_us / np.maximum(d[:, 0][ok], 1)
    for name, key in [("XCC", xcc), ("SE", se), ("SH", sh)]:
        parts = []
        for k in sorted(set(key.tolist())):
            sel = key == k
            parts.append(f"{k}: n {int(sel.sum())} end {q(e_us[sel], 50):.1f} us/item {q(per_item[sel], 50):.1f}")
        print(f"  by {name}: " + "; ".join(parts))
    # the two workgroups sharing a CU
    loc = (xcc << 16) | (se << 8) | (sh << 4) | cu
    same = {}
    for k, e in zip(loc.tolist(), e_us.tolist()):
        same.setdefault(k, []).append(e)
    sizes = [len(v) for v in same.values()]
    print(f"  distinct CUs {len(same)}; workgroups per CU {min(sizes)}-{max(sizes)}")
    items_wg = d[:, 0][ok]
    for k in sorted(set(items_wg.astype(int))):
        sel = items_wg == k
        print(f"    {int(sel.sum())} workgroups with {k} items: end median {q(e_us[sel], 50):.1f} us")
# k_bin's phases (rows 2048+ of the mvs_kernels stamps)
lib.mvs_read_stamps.argtypes = [ctypes.c_void_p]
kbuf = np.zeros(4096 * 16, np.uint64)
lib.mvs_read_stamps(kbuf.ctypes.data)
k0 = kbuf.copy()
ctx.score(c, ref, 0.7, wid)
lib.mvs_read_stamps(kbuf.ctypes.data)
kb = (kbuf - k0).reshape(4096, 16)[2048:].astype(np.float64)
kact = kb[:, 0] > 0
if kact.any():
    print(f"  k_bin: {kact.sum()} workgroups; per workgroup: loads + projection + LDS ranks {kb[kact, 1].mean():.0f}, "
          f"global tile bases + items {kb[kact, 2].mean():.0f}, bucket writes {kb[kact, 3].mean():.0f} cycles")

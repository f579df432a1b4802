import importlib, sys, numpy as np
sys.path.insert(0, '/root/repo')
import bench
pkg = importlib.import_module(bench.PKG_NAME)
rgb, K, R, t = bench.load_scene()
c, ref = pkg.synthetic.candidates(1 << 20, K, R, t, seed=0)
import torch
cx = pkg.MvsContext(rgb, K, R, t)
for wid in (5, 3):
    h0 = cx.exact_hits()
    cx.score(c, ref, 0.7, wid)
    print("wid", wid, "exact-path lanes", cx.exact_hits() - h0)

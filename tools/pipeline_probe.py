"""Probe: sweeps in flight on two streams (two scratch sets) against one
stream, on the bench's dinoRing 2^20 sweep (records, wid 5).  The question:
how much of k_bin / k_score_fix / the scorer's tail hides when the next
sweep's kernels may start on CUs the current sweep's persistent scorer
leaves idle.  MODE=ctx: two MvsContexts (own scratch each); MODE=lib: one
context used from two streams (its scratch slots).
usage: python tools/pipeline_probe.py [steps]"""
import importlib
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
pkg = importlib.import_module(bench.PKG_NAME)
rgb, K, R, t = bench.load_scene()
n = 1 << 20
c, ref = pkg.synthetic.candidates(n, K, R, t, seed=0)
dev = torch.device("cuda:0")
ctx = pkg.MvsContext(rgb, K, R, t, device=0)
mode = os.environ.get("MODE", "lib")
ctx2 = pkg.MvsContext(rgb, K, R, t, device=0) if mode == "ctx" else ctx
tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
xys = [torch.empty((n, 2), dtype=torch.float64, device=dev) for _ in range(2)]
recs = [torch.empty((n, 2), dtype=torch.int64, device=dev) for _ in range(2)]
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def run(k, lanes):
    cxs = [ctx, ctx2]
    for i in range(3):
        for j in range(lanes):
            cxs[j].score_device_rec(tc, tr, xys[j], recs[j], 0.7, 5, stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        j = i % lanes
        cxs[j].score_device_rec(tc, tr, xys[j], recs[j], 0.7, 5, stream=streams[j].cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k


one = run(steps, 1)
two = run(steps, 2)
one2 = run(steps, 1)
m0 = recs[0].cpu().numpy()[:, 0]
m1 = recs[1].cpu().numpy()[:, 0]
print(f"mode {mode}: one stream {one * 1e6:.1f} / {one2 * 1e6:.1f} us per sweep, two streams {two * 1e6:.1f} us "
      f"per sweep; the two record buffers agree: {bool(np.array_equal(m0, m1))}")

"""Device time of mvs_pack_accepted on the bench's 2^20 sweep: 20 back-to-back
packs bracketed by events, on the null stream and on a side stream (the
bench's), and the two kernels' rocprof-free split (count only vs count +
pack, by a cap-0 run that writes the header only).  GPU box only."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = importlib.import_module(bench.PKG_NAME)
rgb, K, R, t = bench.load_scene()
dev = torch.device("cuda:0")
ctx = pkg.MvsContext(rgb, K, R, t, device=0)
n = 1 << 20
c, ref = pkg.synthetic.candidates(n, K, R, t, W=rgb.shape[2], H=rgb.shape[1], seed=0)
tc, tr = torch.from_numpy(np.ascontiguousarray(c)).to(dev), torch.from_numpy(ref).to(dev)
xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
mask = torch.empty((n, 1), dtype=torch.int64, device=dev)
count = torch.empty(n, dtype=torch.int32, device=dev)
ctx.score_device(tc, tr, xy, mask, count, None, 0.7, 5)
torch.cuda.synchronize()
acc = int((count >= 3).sum())
out = torch.empty((acc + acc // 16 + 257, 2), dtype=torch.int64, device=dev)


def timed(stream, cap_out, reps=20):
    for _ in range(3):
        ctx.pack_accepted(0, count, mask, 3, cap_out, stream=stream.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        ctx.pack_accepted(0, count, mask, 3, cap_out, stream=stream.cuda_stream)
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


side = torch.cuda.Stream(dev)
hdr = torch.empty((1, 2), dtype=torch.int64, device=dev)
print(f"accepted {acc}")
print(f"null stream: {timed(torch.cuda.current_stream(dev), out):.2f} us per pack")
print(f"side stream: {timed(side, out):.2f} us per pack")
torch.cuda.set_stream(side)
print(f"side stream (current): {timed(side, out):.2f} us per pack")
print(f"header only (cap 0): {timed(side, hdr):.2f} us per pack")
print(f"null stream, 200 reps: {timed(torch.cuda.current_stream(dev), out, 200):.2f} us per pack")
ctx.close()

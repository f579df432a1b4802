"""A/B the tiled-kernel variants (MVS_VARIANT) in ONE process, interleaved rounds."""
import importlib, os, sys, time
import numpy as np
import torch
sys.path.insert(0, '/root/repo')
import bench
pkg = importlib.import_module(bench.PKG_NAME)
rgb, K, R, t = bench.load_scene()
n = 1 << 20
c_np, ref_np = pkg.synthetic.candidates(n, K, R, t, seed=0)
dev = torch.device("cuda:0")
c = torch.from_numpy(c_np).to(dev); ref = torch.from_numpy(ref_np).to(dev)
variants = [int(v) for v in (sys.argv[1:] or ["0", "1", "2", "3"])]
wid = int(os.environ.get("AB_WID", "5"))
ctxs = {}
for v in variants:
    os.environ["MVS_VARIANT"] = str(v)
    os.environ["MVS_SCORE_KERNEL"] = os.environ.get("AB_KERNEL", "tiled")
    ctxs[v] = pkg.MvsContext(rgb, K, R, t)
stream = torch.cuda.Stream(dev)
torch.cuda.synchronize()
out = {}
for v in variants:
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    mask = torch.empty((n, 1), dtype=torch.int64, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    avg = torch.empty(n, dtype=torch.float64, device=dev)
    out[v] = (xy, mask, cnt, avg)
times = {(v, a): [] for v in variants for a in (True, False)}
with torch.cuda.stream(stream):
    for rnd in range(12):
        for v in variants:
            for with_avg in (True, False):
                xy, mask, cnt, avg = out[v]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                ctxs[v].score_device(c, ref, xy, mask, cnt, avg if with_avg else None, 0.7, wid,
                                     stream=stream.cuda_stream)
                e1.record(stream)
                e1.synchronize()
                if rnd >= 2:
                    times[(v, with_avg)].append(e0.elapsed_time(e1))
base = variants[0]
for v in variants:
    same = torch.equal(out[v][1], out[base][1]) and torch.equal(out[v][2], out[base][2])
    for with_avg in (True, False):
        ts = np.array(times[(v, with_avg)])
        print(f"variant {v} avg={with_avg!s:5}: median {np.median(ts):.4f} ms min {ts.min():.4f} ms "
              f"-> {n / np.median(ts) / 1e6:.0f} M cand/ms*1e3  same_as_{base}={same}")

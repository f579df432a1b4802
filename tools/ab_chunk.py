"""A/B the tiled scorer's work-item size (MVS_TILE_CHUNK) in one process, interleaved."""
import importlib, os, sys
import numpy as np
import torch
sys.path.insert(0, '/root/repo')
import bench
pkg = importlib.import_module(bench.PKG_NAME)
scene = os.environ.get("AB_SCENE", "dino")
if scene == "dino":
    rgb, K, R, t = bench.load_scene()
else:
    rgb, K, R, t = pkg.synthetic.ring_scene(256, 1080, 1920, seed=0)
V, H, W = rgb.shape[:3]
n = 1 << 20
c_np, ref_np = pkg.synthetic.candidates(n, K, R, t, W=W, H=H, seed=0)
dev = torch.device("cuda:0")
c = torch.from_numpy(c_np).to(dev); ref = torch.from_numpy(ref_np).to(dev)
chunks = [int(v) for v in sys.argv[1:]] or [128, 192, 256, 384, 512]
wid = int(os.environ.get("AB_WID", "5"))
ctxs = {}
for ch in chunks:
    os.environ["MVS_TILE_CHUNK"] = str(ch)
    ctxs[ch] = pkg.MvsContext(rgb, K, R, t)
words = (V + 63) // 64
xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
mask = torch.empty((n, words), dtype=torch.int64, device=dev)
cnt = torch.empty(n, dtype=torch.int32, device=dev)
avg = torch.empty(n, dtype=torch.float64, device=dev)
stream = torch.cuda.Stream(dev)
times = {ch: [] for ch in chunks}
ref_out = None
with torch.cuda.stream(stream):
    for rnd in range(10):
        for ch in chunks:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            ctxs[ch].score_device(c, ref, xy, mask, cnt, avg, 0.7, wid, stream=stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            if rnd >= 2:
                times[ch].append(e0.elapsed_time(e1))
            if ref_out is None:
                ref_out = (mask.clone(), cnt.clone())
            else:
                assert torch.equal(mask, ref_out[0]) and torch.equal(cnt, ref_out[1])
for ch in chunks:
    ts = np.array(times[ch])
    print(f"chunk {ch:4d}: median {np.median(ts):.4f} ms  min {ts.min():.4f} ms  -> {n / np.median(ts) / 1e6:.2f} G cand/s")

"""ring256 scoring through the host entry (mvs_score) and the device entry
(mvs_score_device), timed; MVS_LIB selects the library build."""
import faulthandler
import importlib
import os
import sys
import time

import numpy as np

faulthandler.dump_traceback_later(100, exit=True)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module(bench.PKG_NAME)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
dev = torch.device("cuda", 0)
rgb, K, R, t = pkg.synthetic.sphere_scene_device(256, 1080, 1920, seed=0, device=dev)
c, ref = pkg.synthetic.candidates(n, K, R, t, W=1920, H=1080, seed=0)
ctx = pkg.MvsContext(rgb, K, R, t)
print("context ready", flush=True)
for mode in ("device", "host", "host"):
    t0 = time.perf_counter()
    if mode == "device":
        dc = torch.from_numpy(np.ascontiguousarray(c)).to(dev)
        dr = torch.from_numpy(np.ascontiguousarray(ref)).to(dev)
        xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
        mask = torch.empty((n, 4), dtype=torch.int64, device=dev)
        cnt = torch.empty(n, dtype=torch.int32, device=dev)
        avg = torch.empty(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.score_device(dc, dr, xy, mask, cnt, avg, 0.7, 5)
        torch.cuda.synchronize()
        acc = int((cnt >= 3).sum().item())
    else:
        _, _, cnt_h, _ = ctx.score(c, ref, 0.7, 5)
        acc = int((cnt_h >= 3).sum())
    print(f"{mode}: {1e3 * (time.perf_counter() - t0):.1f} ms, accepted {acc}", flush=True)

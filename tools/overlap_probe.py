"""Why does a second-stream copy (the N = 8 all-gather's CU footprint) not
overlap the scorer?  Variants of bench.py's overlap proxy on one GPU:

  base      scoring and comm streams from torch's pool (what bench.py does)
  prio      the comm stream at high priority
  cumask    the scoring stream created with hipExtStreamCreateWithCUMask,
            leaving FREE CUs out of its mask, and the scorer's grid at two
            workgroups per CU of the mask (MVS_SCORER_WGS)
  cumask+prio

Per variant: step time alone (score + 40-B pack), with the copy after each
pack, and the copy alone (32 workgroups, 74 MB).  Run it under
`rocprofv3 --kernel-trace` to read the timeline (tools/overlap_timeline.py).

usage: overlap_probe.py [variants...] [--free K] [--steps S] [--mask-order lo|hi|spread]
"""
import argparse
import ctypes
import importlib
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

PKG_NAME = bench.PKG_NAME


def cu_mask_stream(torch, dev, ncu, free, order):
    """A stream whose kernels run on ncu - free CUs only (bit k = CU k of the
    mask as HIP numbers them); returns (torch ExternalStream, raw handle)."""
    hip = importlib.import_module(PKG_NAME + ".parallel")._hip()   # the runtime torch loaded
    bits = [1] * ncu
    if order == "lo":
        off = list(range(free))
    elif order == "hi":
        off = list(range(ncu - free, ncu))
    else:   # spread: every (ncu // free)-th CU
        off = list(range(0, ncu, max(ncu // free, 1)))[:free]
    for k in off:
        bits[k] = 0
    words = []
    for w in range((ncu + 31) // 32):
        v = 0
        for b in range(32):
            k = 32 * w + b
            if k < ncu and bits[k]:
                v |= 1 << b
        words.append(v)
    arr = (ctypes.c_uint32 * len(words))(*words)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value, device=dev), s.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", default=["base", "prio", "cumask", "cumask+prio"])
    ap.add_argument("--free", type=int, default=16)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--workgroups", type=int, default=32)
    ap.add_argument("--mask-order", default="hi", choices=["lo", "hi", "spread"])
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module(PKG_NAME)
    par = importlib.import_module(PKG_NAME + ".parallel")
    syn = pkg.synthetic
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rgb, K, R, t = bench.load_scene()
    V = rgb.shape[0]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    n = 1 << 20
    c_np, ref_np = syn.candidates(n, K, R, t, seed=0)
    sw = {"c": torch.from_numpy(c_np).to(dev), "ref": torch.from_numpy(ref_np).to(dev),
          "xy": torch.empty((n, 2), dtype=torch.float64, device=dev),
          "rec": torch.empty((n, 2), dtype=torch.int64, device=dev), "off": 0}
    vlb = 3
    print(f"{ncu} CUs; free {a.free} ({a.mask_order}); proxy {a.workgroups} workgroups", flush=True)
    for var in a.variants:
        cum = "cumask" in var
        if cum:
            stream, _ = cu_mask_stream(torch, dev, ncu, a.free, a.mask_order)
            os.environ["MVS_SCORER_WGS"] = str(2 * (ncu - a.free))
        else:
            stream = torch.cuda.Stream(dev)
        try:
            ctx = pkg.MvsContext(rgb, K, R, t, device=0)
        finally:
            os.environ.pop("MVS_SCORER_WGS", None)
        comm = torch.cuda.Stream(dev, priority=-1) if "prio" in var else torch.cuda.Stream(dev)
        ctx.score_device_rec(sw["c"], sw["ref"], sw["xy"], sw["rec"], 0.7, 5, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        acc = int((np.bitwise_count(sw["rec"][:, 0].cpu().numpy().view(np.uint64)) >= vlb).sum())
        cap = acc + acc // 16 + 256
        width = par.points_width(1)
        out = torch.empty((cap + 1, width), dtype=torch.int64, device=dev)
        recv = (7 * (cap + 1) * width * 8 + 15) // 16 * 16
        src = torch.zeros(recv // 8, dtype=torch.int64, device=dev)
        dst = torch.empty_like(src)

        # "pipe": the pack runs on the comm stream too (before the copy), on
        # the sweep's records of the previous step (two record buffers)
        pipe = "pipe" in var
        recs = [sw["rec"], torch.empty_like(sw["rec"])]
        done = [None, None]

        def run(k, with_proxy, proxy_only=False):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for st in range(k):
                rec = recs[st & 1] if pipe else sw["rec"]
                if not proxy_only:
                    if pipe and done[st & 1] is not None:
                        stream.wait_event(done[st & 1])     # the pack two steps back has read rec
                    ctx.score_device_rec(sw["c"], sw["ref"], sw["xy"], rec, 0.7, 5, stream=stream.cuda_stream)
                    if not pipe:
                        ctx.pack_accepted(0, None, rec, vlb, out, stream=stream.cuda_stream, c=sw["c"])
                if with_proxy or pipe:
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    comm.wait_event(ev)
                    if pipe and not proxy_only:
                        ctx.pack_accepted(0, None, rec, vlb, out, stream=comm.cuda_stream, c=sw["c"])
                        done[st & 1] = torch.cuda.Event()
                        done[st & 1].record(comm)
                    if with_proxy:
                        pkg._lib.proxy_copy(dst, src, recv, a.workgroups, comm.cuda_stream)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / k * 1e6

        run(3, True)
        alone = run(a.steps, False)
        both = run(a.steps, True)
        ponly = run(a.steps, True, proxy_only=True)
        print(f"{var:12s} step alone {alone:7.1f} us   with copy {both:7.1f} us   copy alone {ponly:7.1f} us   "
              f"overlap {(alone + ponly - both) / ponly:5.2f} of the copy", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()

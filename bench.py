"""Benchmark: candidate patches NCC-scored per second (BASELINE.json metric).

Headline (BASELINE configs[1]): the real dinoRing
gray stack (48 views x 640x480, data/dinoRing), one expansion sweep = a batch
of 2^20 candidate patches per GPU (reference view, sub-pixel pixel, depth
0.60-0.72 m), every candidate photo-tested against all 48 views with the
reference's 11x11 window (wid=5, MVS2.py:64/69) at MIN_NCC 0.7.  The sweep is
one block of a global candidate queue: rank r scores block r (seed r) of a
queue of N x 2^20 candidates (weak scaling), or with --strong its
shard_range slice of one 2^20 queue.  A step = score the sweep on the GPU
(inputs resident in HBM) + the sweep's exchange (N > 1): the accepted
candidates (|V| >= 3) as 40-B rows [global index, mask word, x, y, z] -- the
accepted 3D points themselves -- packed on the device (one launch, no host
sync) and all-gathered over RCCL on a second stream, overlapping the next
sweep (parallel.PointsExchange).

Beside the headline (rank 0 at N = 1 only, so that the driver's N > 1 runs
stay short):
  roofline     the binding roof of the dominant kernel (k_score_mma) from the
               live kernel time and the per-launch counters of the committed
               rocprofv3 PMC profile (profiles/r05/pmc.json): HBM bytes,
               VALU-busy cycles, MFMA i8 operations; frac <= 1 each
  cold_sweep   scene setup from the resident images (k_build_scene) + the sweep
  secondary    wid 3 (BASELINE config 2's 7x7 window)
  stage        the whole reference stage: DensePointsWithMVS2 on dinoRing +
               tests/golden/seeds_dino.npz with the reference's 100,000-pop cap
               (MVS2.py:321), wall time, reference-equivalent tests/s, phase
               times, rows checked against the oracle fixture's sha256
  ring256      SURVEY 8(d) config 4: 256 views of 1920x1080 (a textured sphere,
               rendered on the GPU so that sweeps accept candidates), 2^20
               candidates per sweep, view-group scorer
  cpu_baseline the oracle (C port of the reference arithmetic) on the host cores,
               and beside it the reference's own single-core Python rate recorded
               at fixture generation (tests/golden/reference_timing.json)

python bench.py [--gpus N --steps K --warmup W --n CANDS --wid 5]
N > 1: either under a launcher (python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N ..., which must start exactly N ranks), or `python bench.py
--gpus N` alone: the process then starts the N ranks itself as children of a
torch.distributed.run subprocess (before touching the GPU), relays rank 0's JSON
line and exits with the children's status.
"""
import argparse
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_NAME = "simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd"
sys.path.insert(0, REPO)

PEAK_HBM = 8.0e12          # MI355X HBM3E, B/s (MI355X_MICROARCH.md)
PEAK_I8 = 5.0e15           # dense i8 MFMA ops/s (2x the 2.5 PF dense bf16; no sparsity)
SIMDS = 1024               # 256 CUs x 4 SIMDs
CLOCK = 2.4e9              # peak engine clock, Hz
# per-launch PMC counters of the scorers (tools/pmc.sh + tools/pmc_json.py):
# this round's profile, else the last round's
PMC_PATH = next((p for p in (os.path.join(REPO, "profiles", r, "pmc.json") for r in ("r06", "r05"))
                 if os.path.exists(p)), os.path.join(REPO, "profiles", "r06", "pmc.json"))
# kernel / score-call timing: HIP and torch events on every TIME_EVERY-th timed
# step (the records cost the stream a few us each: sampled, not every step)
TIME_EVERY = 10


def logical_bytes(V, wid):
    """V*(2w+1)^2 window bytes + 32 B in + 8*ceil(V/64) + 16 B out."""
    return V * (2 * wid + 1) ** 2 + 32 + 8 * ((V + 63) // 64) + 16


def floor_bytes(rgb, xy, ref, wid, n):
    """The unique bytes one scorer launch must move between HBM and the chip,
    from the sweep itself: the candidates the scorer sees are those with a
    valid window whose reference window is not constant (k_bin settles the
    rest), and for them it must read the moment-table rows of their distinct
    pixels (S_b int16 + w binary64 per view at V <= 64, S_b + D int32 at
    V > 64; VP views per row), the gray bytes of their distinct tiles (V views
    x 8 x 16 pixels: the regions' halos overlap the neighbours' and are not
    counted), their bucket entries (8 B) and write their
    records (8 (ceil(V/64) + 1) B).  rgb: (V, H, W, 3) uint8 (host or device); xy, ref:
    device tensors of the sweep.  The windows' constancy is recomputed here
    from integral images of the gray stack (OpenCV's BGR2GRAY weights on the
    RGB data, HarrisFeatures.py:125)."""
    import torch
    V, H, W = rgb.shape[0], rgb.shape[1], rgb.shape[2]
    words = (V + 63) // 64
    vp = 64 * words if V > 64 else 16 * ((V + 15) // 16)
    npx = (2 * wid + 1) ** 2
    q = xy[:, 0].trunc().long()
    r = xy[:, 1].trunc().long()
    ok = (r - wid >= 0) & (r + wid + 1 < H) & (q - wid > 0) & (q + wid + 1 < W)
    q, r, R = q[ok], r[ok], ref[ok].long()
    S = torch.zeros(len(q), dtype=torch.int64, device=xy.device)
    Q = torch.zeros_like(S)
    for v0 in range(0, V, 16):   # the integral images 16 views at a time (bounded memory)
        v1 = min(V, v0 + 16)
        c = torch.as_tensor(np.ascontiguousarray(rgb[v0:v1]) if isinstance(rgb, np.ndarray) else rgb[v0:v1])
        c = c.to(xy.device).int()
        g = ((c[..., 0] * 1868 + c[..., 1] * 9617 + c[..., 2] * 4899 + 8192) >> 14).long()
        del c
        sel = (R >= v0) & (R < v1)
        for src, dst in ((g, S), (g * g, Q)):
            ii = torch.zeros((v1 - v0, H + 1, W + 1), dtype=torch.int64, device=xy.device)
            ii[:, 1:, 1:] = src.cumsum(1).cumsum(2)
            rv, rr, qq = R[sel] - v0, r[sel], q[sel]
            dst[sel] = (ii[rv, rr + wid + 1, qq + wid + 1] - ii[rv, rr - wid, qq + wid + 1]
                        - ii[rv, rr + wid + 1, qq - wid] + ii[rv, rr - wid, qq - wid])
            del ii
        del g
    seen = npx * Q != S * S
    q, r = q[seen], r[seen]
    binned = int(seen.sum())
    pixels = int(torch.unique(r * W + q).numel())
    ntx = (W + 15) // 16
    tiles = int(torch.unique((r // 8) * ntx + q // 16).numel())
    parts = {"tables": pixels * vp * (6 if V > 64 else 10), "gv": tiles * V * 8 * 16,
             "bucket_entries": 8 * binned, "records": 8 * (words + 1) * binned}
    return sum(parts.values()), parts, {"scored_candidates": binned, "of": n, "distinct_pixels": pixels,
                                        "tiles": tiles}


def score(cx, sw, wid, thr, stream, rec=None):
    """One sweep's photo test: records (mvs_score_device_rec, one 16-B store per
    candidate at V <= 64; `rec` overrides the buffer) unless --soa asked for
    the three-array outputs."""
    if sw["rec"] is not None:
        cx.score_device_rec(sw["c"], sw["ref"], sw["xy"], sw["rec"] if rec is None else rec, thr, wid,
                            stream=stream.cuda_stream)
    else:
        cx.score_device(sw["c"], sw["ref"], sw["xy"], sw["mask"], sw["count"], sw["avg"], thr, wid,
                        stream=stream.cuda_stream)


def pack_src(sw, rec=None):
    """(count, mask) arguments of the pack: (None, records) or the arrays."""
    if sw["rec"] is not None:
        return None, (sw["rec"] if rec is None else rec)
    return sw["count"], sw["mask"]


def host_outputs(sw, m=None):
    """(mask uint64 (m, words), count int32 (m,)) of the last sweep, on the host."""
    if sw["rec"] is not None:
        r = sw["rec"][:m].cpu().numpy().view(np.uint64)[:, :-1]
        return r, np.bitwise_count(r).sum(axis=1).astype(np.int32)
    return sw["mask"][:m].cpu().numpy().view(np.uint64), sw["count"][:m].cpu().numpy()


def load_scene():
    from PIL import Image
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "data", "dinoRing", "*.png")))
    rgb = np.stack([np.asarray(Image.open(f).convert("RGB")) for f in files])
    par = os.path.join(REPO, "data", "dinoRing", "dinoR_par.txt")
    K, R, t = [], [], []
    for line in open(par).readlines()[1:]:
        v = [float(x) for x in line.split()[1:]]
        K.append(np.array(v[0:9]).reshape(3, 3))
        R.append(np.array(v[9:18]).reshape(3, 3))
        t.append(np.array(v[18:21]))
    return rgb, np.array(K), np.array(R), np.array(t)


def pmc_entry(scene, V, wid, n, kernel):
    """Per-launch counters of the scorer kernel `kernel` for this
    configuration from the committed PMC profile, or None (counters of
    another kernel never price this one)."""
    if not os.path.exists(PMC_PATH):
        return None
    try:
        for e in json.load(open(PMC_PATH))["entries"]:
            if (e["scene"], e["V"], e["wid"], e["n"]) == (scene, V, wid, n) and kernel + "<" in e["kernel"]:
                return e
    except Exception:
        return None
    return None


def scorer_stats(ctx):
    """MvsContext.scorer_stats(), or zeros from an older A/B library (MVS_LIB)
    without the entry point."""
    try:
        st = ctx.scorer_stats()
    except AttributeError:
        st = {"direct": 0, "overflow": 0, "batches": 0}
    st["exact"] = ctx.exact_hits()
    return st


def direct_path(before, after):
    """Candidates per sweep that k_score_fix re-scored by the direct path
    (the tiled scorer's binary32 guard band + bucket overflow), from two
    MvsContext.scorer_stats() readings."""
    b = max(after["batches"] - before["batches"], 1)
    d = after["direct"] - before["direct"]
    o = after["overflow"] - before["overflow"]
    return {"per_sweep": d / b, "overflow_per_sweep": o / b, "guard_band_per_sweep": (d - o) / b,
            "numpy_order_ncc_per_sweep": (after["exact"] - before["exact"]) / b, "sweeps": b}


def roofline(entry, V, wid, n, kms, kernel, floor):
    """Roofs of the dominant kernel: measured HBM bytes, VALU-busy cycles and
    MFMA i8 operations per launch (PMC) over the live launch time.  The binding
    roof is the one with the largest fraction; each frac <= 1 because a unit
    cannot be busier than its peak.  Beside them the unique-byte floor of a
    launch (floor_bytes): useful_frac = floor / launch time / 8 TB/s, and
    traffic / floor = how much of the counted traffic is re-reads."""
    npx = (2 * wid + 1) ** 2
    fb, fparts, fset = floor
    out = {"kernel": entry["kernel"] if entry else kernel, "kernel_ms": kms,
           "candidates_per_launch": n,
           "floor_bytes": fb, "floor_parts": fparts, "floor_set": fset,
           "useful_GBps": fb / (kms * 1e-3) / 1e9,
           "useful_frac": fb / (kms * 1e-3) / PEAK_HBM,
           "survey_model_bytes_per_candidate": logical_bytes(V, wid),
           "survey_model_note": "SURVEY 8(d) prices a candidate at V (2w+1)^2 + 56 B (every window read "
                                "once per candidate); the scorer stages a tile's region once for all "
                                "its candidates, so that model exceeds the HBM peak by construction "
                                "and is no traffic figure: floor_bytes is"}
    roofs = {}
    useful = 2.0 * V * npx * n        # the window products sum s_R s_v of all V views
    roofs["mfma_useful"] = {"achieved": useful / (kms * 1e-3) / 1e12, "peak": PEAK_I8 / 1e12,
                            "unit": "TOP/s (i8, useful window products)"}
    traffic = None
    if entry:
        c = entry["per_launch"]
        traffic = c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024
        roofs["hbm"] = {"achieved": traffic / (kms * 1e-3) / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                        "bytes_per_launch": traffic,
                        "note": "2 x FETCH_SIZE + WRITE_SIZE: FETCH counts Infinity-Cache (MALL) hits too, "
                                "so on a cache-resident scene this is L2-miss traffic, not DRAM bytes"}
        out["traffic_over_floor"] = traffic / fb
        valu = c["SQ_ACTIVE_INST_VALU"] * 4.0            # quad-cycles -> cycles, summed over SIMDs
        roofs["valu"] = {"achieved": valu / (kms * 1e-3) / 1e9, "peak": SIMDS * CLOCK / 1e9,
                         "unit": "G SIMD-busy-cycles/s",
                         "pmc_self_frac": valu / (SIMDS * c["GRBM_GUI_ACTIVE"] / 8.0)}
        if "SQ_INSTS_VALU_MFMA_I8" in c:
            ops = c["SQ_INSTS_VALU_MFMA_I8"] * 16 * 16 * 64 * 2.0
            roofs["mfma_issued"] = {"achieved": ops / (kms * 1e-3) / 1e12, "peak": PEAK_I8 / 1e12,
                                    "unit": "TOP/s (i8, issued)"}
    for r in roofs.values():
        r["frac"] = r["achieved"] / r["peak"]
    bound = max(roofs, key=lambda k: roofs[k]["frac"])
    b = roofs[bound]
    out.update({"bound": bound, "achieved": b["achieved"], "peak": b["peak"], "unit": b["unit"],
                "frac": b["frac"], "traffic": traffic, "roofs": roofs,
                "source": os.path.relpath(PMC_PATH, REPO) if entry else None})
    return out


def exchange_figures(ctx, sw, V, vlb, accepted, world, stream, thr, wid):
    """The per-sweep exchange's payload and its device pack time (HIP events
    over 20 packs of this rank's scored sweep on the scoring stream), and the
    all-gather each rank receives at N = 8."""
    import torch
    par = importlib.import_module(PKG_NAME + ".parallel")
    words = (V + 63) // 64
    row = 8 * par.points_width(words)
    cap = accepted + accepted // 16 + 256
    out = torch.empty((cap + 1, par.points_width(words)), dtype=torch.int64, device=sw["c"].device)
    pc, pm = pack_src(sw)
    for _ in range(3):
        ctx.pack_accepted(sw["off"], pc, pm, vlb, out, stream=stream.cuda_stream, c=sw["c"])
    # device time: the packs queue up behind ten sweeps' worth of scoring
    # (~1 ms), so the host's submission rate (a ctypes call and a launch per
    # pack, ~15 us) does not pace them
    for _ in range(10):
        score(ctx, sw, wid, thr, stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(20):
        ctx.pack_accepted(sw["off"], pc, pm, vlb, out, stream=stream.cuda_stream, c=sw["c"])
    e1.record(stream)
    e1.synchronize()
    if int(out[0, 0].item()) != accepted:
        raise RuntimeError(f"pack header {int(out[0, 0].item())} != {accepted} accepted")
    # the same pack without the points: 16-B rows [index, mask word]
    out16 = torch.empty((cap + 1, par.points_width(words, points=False)), dtype=torch.int64, device=sw["c"].device)
    for _ in range(10):
        score(ctx, sw, wid, thr, stream)
    e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e2.record(stream)
    for _ in range(20):
        ctx.pack_accepted(sw["off"], pc, pm, vlb, out16, stream=stream.cuda_stream)
    e3.record(stream)
    e3.synchronize()
    if int(out16[0, 0].item()) != accepted:
        raise RuntimeError(f"16-B pack header {int(out16[0, 0].item())} != {accepted} accepted")
    return {"row_bytes": row, "rows_per_rank": accepted, "bytes_per_rank": row * (cap + 1),
            "pack_us": e0.elapsed_time(e1) / 20 * 1e3,
            "pack_us_16B_rows": e2.elapsed_time(e3) / 20 * 1e3,
            "received_per_rank_at_n8_MB": 7 * row * (cap + 1) / 1e6,
            "note": "rows [global index, mask word, x, y, z]: the accepted 3D points themselves; "
                    "pack = mvs_pack_accepted (count + ballot-compacted rows, no host sync), device time "
                    "of 20 packs queued behind ten sweeps of scoring work; the "
                    "all-gather runs on its own stream behind the next sweep (parallel.PointsExchange)"}


def overlap_proxy(ctx, sw, V, vlb, accepted, stream, thr, wid, steps, workgroups=32, comm=None):
    """The N = 8 exchange's footprint beside scoring, on one GPU.
    Each step scores the sweep and packs its accepted rows (40 B) on
    `stream`; the stream `comm` waits for the pack and runs a copy kernel of
    `workgroups` workgroups moving the bytes one rank receives at N = 8
    (RCCL's all-gather is a kernel on a few CUs streaming bytes), overlapping
    the next step.  With the multi-GPU layout `stream` is CU-masked and
    `comm` holds the CUs it leaves out.  Reported: the step (score + pack)
    alone, with the proxy copy too, and the copy alone on `comm`."""
    import torch
    pkg = importlib.import_module(PKG_NAME)
    par = importlib.import_module(PKG_NAME + ".parallel")
    dev = sw["c"].device
    words = (V + 63) // 64
    width = par.points_width(words)
    cap = accepted + accepted // 16 + 256
    recv = (7 * (cap + 1) * width * 8 + 15) // 16 * 16
    src = torch.zeros(recv // 8, dtype=torch.int64, device=dev)
    dst = torch.empty_like(src)
    out = torch.empty((cap + 1, width), dtype=torch.int64, device=dev)
    comm = comm if comm is not None else torch.cuda.Stream(dev)
    def run(k, with_proxy):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st in range(k):
            score(ctx, sw, wid, thr, stream)
            pc, pm = pack_src(sw)
            ctx.pack_accepted(sw["off"], pc, pm, vlb, out, stream=stream.cuda_stream, c=sw["c"])
            if with_proxy:
                ev = torch.cuda.Event()
                ev.record(stream)
                comm.wait_event(ev)
                pkg._lib.proxy_copy(dst, src, recv, workgroups, comm.cuda_stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k

    run(3, True)
    alone = run(steps, False)
    both = run(steps, True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(comm)
    for _ in range(10):
        pkg._lib.proxy_copy(dst, src, recv, workgroups, comm.cuda_stream)
    e1.record(comm)
    e1.synchronize()
    return {"proxy": f"copy kernel of {workgroups} workgroups moving the N = 8 per-rank receive "
                     f"({recv / 1e6:.1f} MB of 40-B rows) on a second stream after each step's pack",
            "step_us_score_pack": alone * 1e6, "step_us_with_proxy": both * 1e6,
            "proxy_alone_us": e0.elapsed_time(e1) / 10 * 1e3, "received_bytes": recv, "workgroups": workgroups}


def launch_ranks(nranks):
    """`bench.py --gpus N` (N > 1) without a launcher: start the N ranks as
    children (python -m torch.distributed.run, one process per GPU, rendezvous
    on 127.0.0.1), forward their output, print rank 0's JSON line as this
    process's only stdout line, and return the exit status (non-zero when any
    rank failed or no line came).  Runs before anything initialises the GPU:
    this process never touches it."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # the ranks' arguments travel in the environment: torch.distributed.run
    # would take some of them (e.g. --n) as abbreviations of its own options
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    env = dict(os.environ, MVS_BENCH_ARGV=json.dumps(sys.argv[1:]))
    line = None
    with subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env) as p:
        for ln in p.stdout:
            if ln.startswith("{") and '"metric"' in ln:
                line = ln.strip()
            else:
                sys.stderr.write(ln)
                sys.stderr.flush()
        rc = p.wait()
    if line is not None:
        print(line, flush=True)
    if rc == 0 and line is None:
        print(f"bench.py: the {nranks} ranks exited without a result line", file=sys.stderr)
        rc = 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group backend for N > 1 (nccl = RCCL over xGMI; gloo only "
                         "to rehearse the multi-rank path with several ranks on one GPU)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=1 << 20, help="candidates per GPU per sweep")
    ap.add_argument("--strong", action="store_true",
                    help="one queue of --n candidates split over the ranks (default: --n per rank)")
    ap.add_argument("--wid", type=int, default=5)
    ap.add_argument("--thr", type=float, default=0.7)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=500000,
                    help="candidates the single-threaded oracle scores (~10 s)")
    ap.add_argument("--secondary-wid", type=int, default=3)
    ap.add_argument("--no-stage", action="store_true", help="skip the full-stage secondary")
    ap.add_argument("--no-ring", action="store_true", help="skip the ring256 secondary")
    ap.add_argument("--no-overlap", action="store_true", help="skip the exchange overlap proxy")
    ap.add_argument("--soa", action="store_true",
                    help="score into the three output arrays (mask, count, avg) instead of one record per candidate")
    ap.add_argument("--comm-cus", type=int, default=16,
                    help="N > 1 (and the N = 1 with-pack baseline): CUs left to the all-gather's kernel "
                         "(0: none)")
    ap.add_argument("--comm-layout", choices=["mask", "grid"], default="grid",
                    help="how --comm-cus are kept free: a CU-masked scoring stream (mask) or the "
                         "persistent scorer's grid at two workgroups per remaining CU (grid)")
    ap.add_argument("--pack-on-comm", action="store_true",
                    help="N > 1: pack on the exchange's stream (the CUs the masked scoring stream leaves "
                         "out), overlapping the next sweep (default: on the scoring stream, after the sweep)")
    ap.add_argument("--scene", choices=["dino", "ring256"], default="dino",
                    help="headline scene (ring256: config 4 as the headline, for profiling)")
    argv = json.loads(os.environ["MVS_BENCH_ARGV"]) if "MVS_BENCH_ARGV" in os.environ else None
    a = ap.parse_args(argv)
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.pack_on_comm and a.soa:
        # the SoA outputs are single-buffered: the next sweep would overwrite
        # count / mask while the comm stream's pack still reads them
        raise SystemExit("--pack-on-comm needs the record outputs (not --soa)")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # no launcher: this process starts the ranks and never touches the GPU
        sys.exit(launch_ranks(a.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)")
    ndev = torch.cuda.device_count()
    if world > 1 and a.backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, {ndev} visible "
                         "(--backend gloo rehearses several ranks on one GPU)")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != a.gpus:
            raise SystemExit(f"bench.py: process group of {dist.get_world_size()} ranks, --gpus {a.gpus}")
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": local,
          "pci_bus_id": getattr(props, "pci_bus_id", None), "name": props.name}
    ranks_info = [me]
    if world > 1:
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, me)
    pkg = importlib.import_module(PKG_NAME)
    par = importlib.import_module(PKG_NAME + ".parallel")
    syn = pkg.synthetic

    def make_scene(which):
        if which == "dino":
            return load_scene()
        return syn.sphere_scene_device(256, 1080, 1920, seed=0, device=dev)

    rgb, K, R, t = make_scene(a.scene)
    V, H, W = rgb.shape[0], rgb.shape[1], rgb.shape[2]
    ctx = pkg.MvsContext(rgb, K, R, t, device=local)
    vlb = 3 if V > 2 else 2
    stream = torch.cuda.Stream(dev)          # the scoring kernels run on THIS stream
    torch.cuda.synchronize()
    torch.cuda.set_stream(stream)

    def sweep_inputs(ctx_V, Kc, Rc, tc, Wc, Hc, n_local, strong):
        """This rank's block of the global candidate queue (device tensors)."""
        if strong:
            b, e = par.shard_range(a.n, rank, world)
            c_np, ref_np = syn.candidates(a.n, Kc, Rc, tc, W=Wc, H=Hc, seed=0)
            c_np, ref_np, off = c_np[b:e], ref_np[b:e], b
        else:
            c_np, ref_np = syn.candidates(n_local, Kc, Rc, tc, W=Wc, H=Hc, seed=rank)
            off = rank * n_local
        n = len(ref_np)
        return {"c_np": c_np, "ref_np": ref_np, "off": off, "n": n,
                "c": torch.from_numpy(np.ascontiguousarray(c_np)).to(dev),
                "ref": torch.from_numpy(np.ascontiguousarray(ref_np)).to(dev),
                "xy": torch.empty((n, 2), dtype=torch.float64, device=dev),
                "mask": torch.empty((n, (ctx_V + 63) // 64), dtype=torch.int64, device=dev),
                "count": torch.empty(n, dtype=torch.int32, device=dev),
                "rec": None if a.soa else torch.empty((n, (ctx_V + 63) // 64 + 1), dtype=torch.int64, device=dev),
                "avg": torch.empty(n, dtype=torch.float64, device=dev)}

    def timed(cx, sw, wid, steps, warmup, exchange=True, rebuild=False, st=None):
        """steps timed sweeps on stream st (default: the scoring stream) ->
        (wall s (max over ranks), kernel ms per launch, score-call ms, records
        exchanged in the last step)."""
        got = {"n": 0}
        st = st or stream
        ex = sw.get("exch") if exchange else None

        def step(evs=None):
            rec = None
            if ex is not None and ex.pack_on_comm and sw["rec"] is not None:
                # two record buffers: sweep k+1 scores into one while the comm
                # stream packs sweep k's from the other
                b = ex.posted & 1
                rec = sw["recs"][b]
                # a cross-stream wait costs the scoring stream ~18 us of dead
                # time (profiles/r05/r5c_masked_pack_on_comm_timeline.txt):
                # enqueue it only while the pack two sweeps back is still running
                if ex.consumed(b) is not None and not ex.consumed(b).query():
                    st.wait_event(ex.consumed(b))
            if evs is not None:
                evs[0].record(st)
            if rebuild:
                cx.rebuild(stream=st.cuda_stream)
            score(cx, sw, wid, a.thr, st, rec)
            if evs is not None:
                evs[1].record(st)
            if ex is not None:
                # pack (device, no host sync) + at N > 1 the all-gather on the
                # exchange's own stream, overlapping the next sweep
                # (parallel.PointsExchange); at N = 1 the pack alone
                ex.post(sw["off"], *pack_src(sw, rec), vlb, stream=st, c=sw["c"])

        for _ in range(warmup):
            step()
        # event pairs (the scorer's HIP events and the score call's torch events)
        # on every TIME_EVERY-th step only: each record costs a few us of stream time
        timed_steps = list(range(0, steps, TIME_EVERY))
        evs = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for k in timed_steps}
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        cx.kernel_timing(True, every=TIME_EVERY)   # HIP events around the dominant kernel, on its stream
        t0 = time.perf_counter()
        for k in range(steps):
            step(evs.get(k))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        cx.kernel_timing(False)
        kt, kl = cx.kernel_time()
        if kl != len(timed_steps) or kt <= 0.0:
            raise RuntimeError(f"kernel timing recorded {kl} launches / {kt} ms for {len(timed_steps)} timed steps")
        pms = sum(e0.elapsed_time(e1) for e0, e1 in evs.values()) / len(evs)
        if ex is not None:
            got["n"] = int(sum(ex.accepted()))    # every rank's rows arrived, none over capacity / failed
        if world > 1:
            tt = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        return dt, kt / kl, pms, got["n"]

    sw = sweep_inputs(V, K, R, t, W, H, a.n, a.strong)
    n = sw["n"]
    if sw["rec"] is not None:
        sw["recs"] = [sw["rec"], torch.empty_like(sw["rec"])]
    # the multi-GPU step's layout: scoring on a CU-masked stream
    # (all CUs but --comm-cus), the scorer's grid at two workgroups per kept
    # CU, and the pack + all-gather on the exchange's stream, where they find
    # the free CUs instead of queueing behind the persistent scorer
    mstream, kept, cstream, cowner, owners = stream, None, None, None, []
    if a.comm_cus > 0 and (world > 1 or rank == 0):
        if a.comm_layout == "mask":
            # the streams' owners (parallel.MaskedStream): closed at the end,
            # or at exit by their atexit hook
            mowner = par.cu_masked_stream(dev, a.comm_cus)
            cowner = par.cu_masked_stream(dev, a.comm_cus, complement=True)
            owners = [mowner, cowner]
            mstream, kept, cstream = mowner.stream, mowner.cus, cowner.stream
        else:
            kept = torch.cuda.get_device_properties(dev).multi_processor_count - a.comm_cus

    def masked(on):
        ctx.set_scorer_grid(2 * kept if on and kept else 0)

    pack_on_comm = a.pack_on_comm
    if world > 1:
        # exchange capacity: this sweep's accepted count (one untimed score),
        # the maximum over ranks plus a margin (rows of every rank are equal-sized)
        score(ctx, sw, a.wid, a.thr, stream)
        torch.cuda.synchronize()
        kk = torch.tensor([int((host_outputs(sw)[1] >= vlb).sum())], dtype=torch.int64, device=dev)
        dist.all_reduce(kk, op=dist.ReduceOp.MAX)
        cap = int(kk.item()) + int(kk.item()) // 16 + 256
        sw["exch"] = par.PointsExchange(ctx, (V + 63) // 64, cap, dev, pack_on_comm=pack_on_comm,
                                        comm_stream=cowner if pack_on_comm else None)
        masked(True)
    total_n = a.n if a.strong else a.n * world
    st0 = scorer_stats(ctx)
    dt, kms, pms, gathered = timed(ctx, sw, a.wid, a.steps, a.warmup, st=mstream if world > 1 else stream)
    direct = direct_path(st0, scorer_stats(ctx))
    masked(False)
    value = total_n * a.steps / dt
    accepted = int((host_outputs(sw)[1] >= vlb).sum())
    acc_ranks = [accepted]
    if world > 1:
        acc_ranks = [None] * world
        dist.all_gather_object(acc_ranks, accepted)
    kernel_name = ctx.timed_kernel()
    solo = rank == 0 and world == 1
    scaling_base = None
    if solo:
        # the N = 1 step with the N > 1 step's device work minus the gather:
        # score + the 40-B point pack (PointsExchange at world 1), so that a
        # 1 -> N comparison can also be made on the same device work
        cap1 = accepted + accepted // 16 + 256
        sw["exch"] = par.PointsExchange(ctx, (V + 63) // 64, cap1, dev, pack_on_comm=pack_on_comm,
                                        comm_stream=cowner if pack_on_comm else None)
        masked(True)
        pdt, _, _, packed = timed(ctx, sw, a.wid, a.steps, a.warmup, st=mstream)
        masked(False)
        del sw["exch"]
        if packed != accepted:
            raise RuntimeError(f"N = 1 pack: {packed} rows != {accepted} accepted")
        scaling_base = {"step_ms_with_pack": pdt / a.steps * 1e3, "value_with_pack": n * a.steps / pdt,
                        "step_ms_score_only": dt / a.steps * 1e3,
                        "layout": ((f"scoring on {kept} of {kept + a.comm_cus} CUs (CU-masked stream), "
                                    if a.comm_layout == "mask" else
                                    f"scorer grid {2 * kept} (two workgroups on {kept} CUs' worth), ") if kept else
                                   "scoring on every CU, ") +
                                  ((f"pack on the exchange's stream ({a.comm_cus} CUs)" if kept else
                                    "pack on the exchange's stream") if pack_on_comm else
                                   "pack on the scoring stream, the gather's CUs left free"),
                        "note": "`value` at N = 1 is the scoring step alone (no exchange exists on one GPU); "
                                "at N > 1 a step adds the 40-B point pack and the all-gather (overlapped "
                                "with the next sweep). value_with_pack is the N = 1 step with the pack"}

    out = {
        "metric": ("candidate patches/sec NCC-scored (640×480, 48 views) at 1/2/4/8 MI355X; % HBM roofline"
                   if a.scene == "dino" else
                   "candidate patches/sec NCC-scored (1920×1080, 256 views, synthetic) at 1/2/4/8 MI355X"),
        "value": value,
        "unit": "candidates/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if a.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("real dinoRing images (data/dinoRing)" if a.scene == "dino" else
                 "synthetic textured sphere rendered on the GPU (seed 0)") +
                " + synthetic candidate patches (global queue, block per rank)",
        "config": {"workload": f"{'dinoRing' if a.scene == 'dino' else 'sphere ring'} {V}x{W}x{H}, "
                               f"one expansion sweep of {n} candidates per GPU, "
                               f"{2 * a.wid + 1}x{2 * a.wid + 1} NCC (wid={a.wid}) vs all views, "
                               f"MIN_NCC {a.thr}" +
                               (", accepted points (index, view mask, x y z) packed and all-gathered"
                                if world > 1 else ", one GPU (no exchange)"),
                   "global_batch": total_n, "wid": a.wid, "views": V,
                   "outputs": ("per candidate: xy + mask, count, avg arrays" if a.soa else
                               "per candidate: xy + one record [mask word, avg] (|V| = popcount)"),
                   "parallelism": (f"candidate-queue shards x{world} ({'RCCL' if a.backend == 'nccl' else 'gloo'} "
                                   f"all-gather of accepted points)" if world > 1 else "single GPU")},
        "ranks_seen": len(ranks_info),
        "backend": (a.backend if world > 1 else None),
        "ranks": ranks_info,
        "accepted_per_rank": acc_ranks,
        "scaling_baseline": scaling_base,
        "kernel": kernel_name,
        "kernel_timing": f"HIP events around the scorer on every {TIME_EVERY}th timed step",
        "score_call_ms": pms,
        "accepted_per_sweep": accepted,
        "gathered_records": gathered,
        "direct_path": direct,
        "exchange": exchange_figures(ctx, sw, V, vlb, accepted, world, stream, a.thr, a.wid),
    }
    out["roofline"] = roofline(pmc_entry(a.scene, V, a.wid, n, kernel_name), V, a.wid, n, kms, kernel_name,
                               floor_bytes(rgb, sw["xy"], sw["ref"], a.wid, n))
    if solo and not a.no_overlap:
        # the multi-GPU layout: scoring on the CU-masked stream, the pack and
        # the proxy of RCCL's all-gather on the CUs it leaves out
        masked(True)
        try:
            ov = overlap_proxy(ctx, sw, V, vlb, accepted, mstream, a.thr, a.wid, max(a.steps // 2, 10),
                               comm=cstream)
        finally:
            masked(False)
        ov["layout"] = ((f"scoring + pack on {kept} CUs (CU-masked stream), copy on the other {a.comm_cus}"
                         if a.comm_layout == "mask" else
                         f"scorer grid {2 * kept}, copy on a second stream") if kept else
                        "scoring and exchange on every CU")
        # for comparison: one unmasked stream each (the copy then competes
        # for the CUs the persistent scorer holds)
        ov["unmasked"] = {k: v for k, v in overlap_proxy(
            ctx, sw, V, vlb, accepted, stream, a.thr, a.wid, max(a.steps // 2, 10)).items() if "_us" in k}
        out["exchange"]["overlap_proxy"] = ov

    if solo:
        # cold sweep: scene setup from the resident images + the sweep
        steps_c = max(a.steps // 5, 5)
        cdt, _, cpms, _ = timed(ctx, sw, a.wid, steps_c, 1, exchange=False, rebuild=True)
        out["cold_sweep"] = {"value": n * steps_c / cdt, "unit": "candidates/s",
                             "ms_per_step": cdt / steps_c * 1e3, "setup_plus_score_call_ms": cpms,
                             "note": "k_build_scene (RGB -> gray stack + signed view-major copy) "
                                     "before every sweep; the warm figure is `value`"}
        if a.secondary_wid and a.secondary_wid != a.wid:
            s2 = max(a.steps // 2, 5)
            st0 = scorer_stats(ctx)
            dt2, kms2, pms2, _ = timed(ctx, sw, a.secondary_wid, s2, 2, exchange=False)
            out["secondary"] = {"wid": a.secondary_wid, "value": n * s2 / dt2, "kernel_ms": kms2,
                                "score_call_ms": pms2, "direct_path": direct_path(st0, scorer_stats(ctx)),
                                "roofline": roofline(pmc_entry(a.scene, V, a.secondary_wid, n, kernel_name), V,
                                                     a.secondary_wid, n, kms2, kernel_name,
                                                     floor_bytes(rgb, sw["xy"], sw["ref"], a.secondary_wid, n))}

    if solo and a.scene == "dino" and not a.no_stage:
        sd = dict(np.load(os.path.join(REPO, "tests", "golden", "seeds_dino.npz")))
        fx = json.load(open(os.path.join(REPO, "tests", "golden", "stage_oracle_cap100000.json")))
        ctx.stage(sd["track_off"], sd["obs_view"], sd["obs_xy"], cell_size=2, scale=10.0, wid=5,
                  max_pops=2000)                                       # warm
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            ini, allp, st = ctx.stage(sd["track_off"], sd["obs_view"], sd["obs_xy"], cell_size=2,
                                      scale=10.0, wid=5, max_pops=100000)
            walls.append(time.perf_counter() - t0)
        ok = (hashlib.sha256(np.ascontiguousarray(ini, "<f8").tobytes()).hexdigest() == fx["sha256_initial"]
              and hashlib.sha256(np.ascontiguousarray(allp, "<f8").tobytes()).hexdigest() == fx["sha256_all"])
        w = min(walls)
        out["stage"] = {"workload": "DensePointsWithMVS2 (MVS2.py:176-295) on dinoRing + seeds_dino.npz, "
                                    "100,000 pops (MVS2.py:321), wid 5, cell 2, scale 10",
                        "wall_s": w, "wall_s_runs": walls, "pops": st["pops"],
                        "reference_equivalent_tests": st["tests"],
                        "tests_per_s": st["tests"] / w, "gpu_scored_candidates": st["scored"],
                        "sweeps": st["sweeps"], "patches": len(allp), "initial_patches": len(ini),
                        "phases_s": st["times"], "rows_match_oracle_fixture": bool(ok)}

    if solo and a.scene == "dino" and not a.no_ring:
        rrgb, rK, rR, rt = make_scene("ring256")
        rV, rH, rW = rrgb.shape[:3]
        rctx = pkg.MvsContext(rrgb, rK, rR, rt, device=local)
        rsw = sweep_inputs(rV, rK, rR, rt, rW, rH, a.n, False)
        s3 = max(a.steps // 5, 5)
        rdt, rkms, rpms, _ = timed(rctx, rsw, a.wid, s3, 2, exchange=False)
        out["ring256"] = {"workload": f"SURVEY 8(d) config 4: {rV} views x {rW}x{rH} (textured sphere), "
                                      f"{rsw['n']} candidates per sweep, wid {a.wid}, MIN_NCC {a.thr}",
                          "value": rsw["n"] * s3 / rdt, "unit": "candidates/s", "kernel": rctx.timed_kernel(),
                          "kernel_ms": rkms, "score_call_ms": rpms,
                          "accepted_per_sweep": int((host_outputs(rsw)[1] >= 3).sum()),
                          "roofline": roofline(pmc_entry("ring256", rV, a.wid, rsw["n"], rctx.timed_kernel()), rV,
                                               a.wid, rsw["n"], rkms, rctx.timed_kernel(),
                                               floor_bytes(rrgb, rsw["xy"], rsw["ref"], a.wid, rsw["n"]))}
        rctx.close()
        del rrgb

    if solo and not a.no_cpu_baseline:
        from oracle import oracle as orc
        scene = orc.Scene(rgb, K, R, t)
        m = min(a.cpu_sample * 48 // V, n)     # ~10 s of single-core work
        t0 = time.perf_counter()
        oxy, omask, ocount, _ = scene.score_batch(sw["c_np"][:m], sw["ref_np"][:m], a.thr, a.wid, nthreads=1)
        cdt = time.perf_counter() - t0
        ncores = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "0") or 10**6))
        t0 = time.perf_counter()
        scene.score_batch(sw["c_np"][:m], sw["ref_np"][:m], a.thr, a.wid, nthreads=ncores)
        cdt_all = time.perf_counter() - t0
        # the sample doubles as a parity spot check of the measured kernel
        score(ctx, sw, a.wid, a.thr, stream)
        torch.cuda.synchronize()
        mask_gpu, cnt_gpu = host_outputs(sw, m)
        out["cpu_baseline"] = {
            "value": m / cdt, "unit": "candidates/s", "cores": 1, "kind": "port",
            "sample": f"first {m} of the rank-0 sweep (same candidates, wid={a.wid}), "
                      f"oracle/mvs_oracle.c or_score_batch single-threaded, {cdt:.1f} s",
            "value_all_cores": m / cdt_all, "cores_all": ncores,
            "parity_on_sample": bool(np.array_equal(cnt_gpu, ocount) and
                                     np.array_equal(mask_gpu, omask))}
        # the reference itself (CPython, single thread): its recorded wall time
        # for the longest unfiltered fixture run and the photo tests that run
        # performed (tests/golden/gen_ref_timing.py)
        rt = json.load(open(os.path.join(REPO, "tests", "golden", "reference_timing.json")))
        run = max((r for r in rt["runs"] if "filter" not in r["fixture"]), key=lambda r: r["photo_tests"])
        out["cpu_baseline"]["reference_python"] = {
            "value": run["photo_tests_per_s"], "unit": "candidates/s", "cores": 1, "kind": "reference",
            "sample": f"DensePointsWithMVS2 on dinoRing + seeds_dino.npz to {run['pops']} pops: "
                      f"{run['photo_tests']} photo tests (MVS2.py:255 + :362) in {run['ref_seconds']:.0f} s",
            "provenance": "build container (8-core Xeon), 1 core, measured at fixture generation "
                          f"(tests/golden/gen_golden.py; {run['fixture']}); the reference does not travel "
                          "to the GPU box"}
        if not out["cpu_baseline"]["parity_on_sample"]:
            print("WARNING: GPU/oracle mismatch on the cpu-baseline sample", file=sys.stderr)
    else:
        out["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(out))
    sw.pop("exch", None)
    for o in owners:
        o.close()
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()

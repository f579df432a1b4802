"""Streams, scorer grids and the exchange's comm-stream pack:

* a CU-masked stream (parallel.MaskedStream) used for a score and a pack and
  never closed by the program: the process must still exit cleanly (the
  atexit hook retires it before the runtime's teardown; the round-5 SIGSEGV
  in __cxa_finalize);
* a stream the context has used, retired (mvs_stream_retiring) and
  destroyed, then calls on the context's own stream and on a new stream;
* the persistent scorer held to a reduced grid (mvs_set_scorer_grid): 37
  workgroups on a dense batch (implicit items, the static first items b and
  b + grid, claims from 2 x grid on), and a grid larger than half the work
  items (most workgroups' second static item past the end);
* PointsExchange(pack_on_comm=True) at world 1 over several posts, each
  against parallel.pack_accepted_reference.
Every result is checked against the oracle (oracle/mvs_oracle.c).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG_NAME, REPO, bench_candidates

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pkg, dino):
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    rgb, K, R, t = dino
    c = pkg.MvsContext(rgb, K, R, t, device=0)
    yield c
    c.close()


def _outputs(rec):
    r = rec.cpu().numpy()
    return r[:, 0].view(np.uint64), np.bitwise_count(r[:, 0].view(np.uint64)).astype(np.int32)


EXIT_SCRIPT_SCORE_ONLY = r"""
import sys, numpy as np, torch, importlib
sys.path.insert(0, {repo!r}); sys.path.insert(0, {golden!r})
from make_seeds import load_dino
pkg = importlib.import_module({pkg!r})
par = importlib.import_module({pkg!r} + ".parallel")
imgs, K, R, t = load_dino({data!r})
ctx = pkg.MvsContext(np.stack(imgs), K, R, t, device=0)
ms = par.cu_masked_stream("cuda:0", 16)
c, ref = pkg.synthetic.candidates(1 << 16, K, R, t, seed=3)
dev = torch.device("cuda:0")
tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
xy = torch.empty((len(ref), 2), dtype=torch.float64, device=dev)
rec = torch.empty((len(ref), 2), dtype=torch.int64, device=dev)
ctx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=ms.cuda_stream)
ms.stream.synchronize()
print("scored", flush=True)
"""

EXIT_SCRIPT = r"""
import sys, numpy as np, torch, importlib
sys.path.insert(0, {repo!r}); sys.path.insert(0, {golden!r})
from make_seeds import load_dino
pkg = importlib.import_module({pkg!r})
par = importlib.import_module({pkg!r} + ".parallel")
imgs, K, R, t = load_dino({data!r})
ctx = pkg.MvsContext(np.stack(imgs), K, R, t, device=0)
ms = par.cu_masked_stream("cuda:0", 16)
cs = par.cu_masked_stream("cuda:0", 16, complement=True)
c, ref = pkg.synthetic.candidates(1 << 16, K, R, t, seed=3)
dev = torch.device("cuda:0")
tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
xy = torch.empty((len(ref), 2), dtype=torch.float64, device=dev)
rec = torch.empty((len(ref), 2), dtype=torch.int64, device=dev)
ctx.set_scorer_grid(2 * ms.cus)
ex = par.PointsExchange(ctx, 1, len(ref), dev, pack_on_comm=True, comm_stream=cs)
for _ in range(3):
    ctx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=ms.cuda_stream)
    ex.post(0, None, rec, 3, stream=ms.stream, c=tc)
print("accepted", ex.accepted()[0], flush=True)
# no close(), no destroy_stream, no ctx.close(): the atexit hooks release them
"""


@pytest.mark.parametrize("script", ["score_only", "score_and_pack"])
def test_masked_stream_exit_without_close(dino, script):
    """A masked scoring stream (and a masked comm stream for the exchange's
    pack) left open at exit: rc 0, no signal."""
    code = (EXIT_SCRIPT_SCORE_ONLY if script == "score_only" else EXIT_SCRIPT).format(
        repo=REPO, golden=os.path.join(REPO, "tests", "golden"), pkg=PKG_NAME,
        data=os.path.join(REPO, "data", "dinoRing"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert ("scored" if script == "score_only" else "accepted") in p.stdout


def test_stream_retiring_then_other_streams(pkg, ctx, dino, oracle_scene):
    """Score on a masked stream, retire and destroy it (MaskedStream.close ->
    mvs_stream_retiring), then score on a new torch stream and on the
    context's own stream: all three bit-exact vs the oracle."""
    import importlib
    import torch
    par = importlib.import_module(pkg.__name__ + ".parallel")
    rgb, K, R, t = dino
    n = 1 << 15
    c, ref = bench_candidates(n, K, R, t, seed=21)
    oxy, omask, ocount, _ = oracle_scene.score_batch(c, ref, 0.7, 5, nthreads=8)
    dev = torch.device("cuda:0")
    tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    rec = torch.empty((n, 2), dtype=torch.int64, device=dev)
    with par.cu_masked_stream(dev, 16) as ms:
        torch.cuda.synchronize()
        ctx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=ms.cuda_stream)
        ms.stream.synchronize()
        m, cnt = _outputs(rec)
        assert np.array_equal(m, omask[:, 0]) and np.array_equal(cnt, ocount)
    s = torch.cuda.Stream(dev)
    rec.fill_(-1)
    torch.cuda.synchronize()
    ctx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=s.cuda_stream)
    s.synchronize()
    m, cnt = _outputs(rec)
    assert np.array_equal(m, omask[:, 0]) and np.array_equal(cnt, ocount)
    hxy, hmask, hcount, _ = ctx.score(c, ref, 0.7, 5)   # the context's own stream
    assert np.array_equal(hmask, omask) and np.array_equal(hcount, ocount) and np.array_equal(hxy, oxy)


@pytest.mark.parametrize("case", ["dense_grid37", "sparse_grid400"])
def test_scorer_grid_reduced(pkg, ctx, dino, oracle_scene, case):
    """k_score_tab held to a smaller grid (the multi-GPU layouts do this):
    dense batch at 37 workgroups (implicit items; workgroup b starts with
    items b and b + 37, the queue hands out 74...), and a batch crowded into
    the image's top-left 200 x 100 pixels (~170 tiles, items from
    k_item_scan) at 400 workgroups, more than half the work items; bit-exact
    vs the oracle."""
    import torch
    rgb, K, R, t = dino
    if case == "dense_grid37":
        n, grid = 1 << 18, 37
        c, ref = bench_candidates(n, K, R, t, seed=31)
    else:
        n, grid = 1 << 16, 400
        c, ref = bench_candidates(n, K, R, t, seed=32, W=200, H=100)
    oxy, omask, ocount, oavg = oracle_scene.score_batch(c, ref, 0.7, 5, nthreads=16)
    dev = torch.device("cuda:0")
    tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    rec = torch.empty((n, 2), dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    try:
        ctx.set_scorer_grid(grid)
        for _ in range(2):   # the counters the first batch leaves behind serve the second
            rec.fill_(-1)
            ctx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=s.cuda_stream)
            s.synchronize()
            m, cnt = _outputs(rec)
            assert np.array_equal(m, omask[:, 0]) and np.array_equal(cnt, ocount)
            assert np.allclose(rec.cpu().numpy()[:, 1].view(np.float64), oavg, rtol=0, atol=1e-12)
            assert np.array_equal(xy.cpu().numpy(), oxy)
    finally:
        ctx.set_scorer_grid(0)


def test_points_exchange_pack_on_comm_world1(pkg, ctx, dino):
    """PointsExchange(pack_on_comm=True) at world 1: four sweeps posted back
    to back on a scoring stream, alternating two record buffers as bench.py
    does (a buffer is rewritten only after consumed(b)); every buffer's rows
    equal pack_accepted_reference of its own sweep."""
    import importlib
    import torch
    par = importlib.import_module(pkg.__name__ + ".parallel")
    rgb, K, R, t = dino
    n = 1 << 17
    dev = torch.device("cuda:0")
    sweeps = [bench_candidates(n, K, R, t, seed=40 + k) for k in range(4)]
    s = torch.cuda.Stream(dev)
    ex = par.PointsExchange(ctx, 1, n, dev, pack_on_comm=True)
    recs = [torch.empty((n, 2), dtype=torch.int64, device=dev) for _ in range(2)]
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    keep = []
    for k, (c, ref) in enumerate(sweeps):
        b = ex.posted & 1
        if ex.consumed(b) is not None:
            s.wait_event(ex.consumed(b))
        tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
        keep.append((tc, tr))
        torch.cuda.synchronize()
        ctx.score_device_rec(tc, tr, xy, recs[b], 0.7, 5, stream=s.cuda_stream)
        assert ex.post(1000 * k, None, recs[b], 3, stream=s, c=tc) == b
        if k >= 1:
            # the previous sweep's buffer: packed while this sweep scored
            pb = b ^ 1
            blk = ex.check(pb)
            pc, _ = sweeps[k - 1]
            exp = torch.zeros((n + 1, par.points_width(1)), dtype=torch.int64)
            torch.cuda.synchronize()
            par.pack_accepted_reference(1000 * (k - 1), None, prev_rec, 3, exp, torch.from_numpy(pc))
            acc = int(exp[0, 0])
            assert acc > 1000
            got = blk[0].cpu()
            assert torch.equal(got[0], exp[0]) and torch.equal(par.sort_rows(got[1:1 + acc]), exp[1:1 + acc])
        s.synchronize()
        prev_rec = recs[b].cpu()
    blk = ex.check()
    exp = torch.zeros((n + 1, par.points_width(1)), dtype=torch.int64)
    par.pack_accepted_reference(3000, None, prev_rec, 3, exp, torch.from_numpy(sweeps[3][0]))
    got, acc = blk[0].cpu(), int(exp[0, 0])
    assert torch.equal(got[0], exp[0]) and torch.equal(par.sort_rows(got[1:1 + acc]), exp[1:1 + acc])


def _skewed_candidates(n, K, R, t, seed):
    """n candidates crowded onto two pixel tiles (most overflow the buckets)."""
    rng = np.random.default_rng(seed)
    ref = rng.integers(0, 48, n).astype(np.int32)
    x = np.where(rng.random(n) < 0.5, 300.0, 333.0) + rng.random(n) * 15.9
    y = 200 + rng.random(n) * 7.9
    z = rng.uniform(0.6, 0.72, n)
    Kinv = np.linalg.inv(K)
    ray = np.einsum("nij,nj->ni", Kinv[ref], np.stack([x, y, np.ones(n)], 1))
    c = np.einsum("nji,nj->ni", R[ref], z[:, None] * ray - t[ref].reshape(n, 3))
    return np.ascontiguousarray(c), ref


def test_counter_sets_alternate_across_batch_kinds(pkg, dino, oracle_scene):
    """The tiled scorer's two counter sets (parities): each batch's k_bin
    zeroes the previous batch's set, so no kernel after the scorer zeroes
    anything.  A fresh context runs, on two streams in turn, a skewed batch
    (bucket overflow onto the direct path's list), a dense batch (implicit
    items), a sparse one (k_item_scan), a small one (the direct kernel: no
    counters touched) and the dense and skewed ones again: every output
    equals the oracle's, and the statistics count the overflow of the skewed
    batches only."""
    import torch
    rgb, K, R, t = dino
    dev = torch.device("cuda:0")
    batches = {
        "skewed": _skewed_candidates(1 << 15, K, R, t, seed=51),
        "dense": bench_candidates(1 << 18, K, R, t, seed=52),
        "sparse": bench_candidates(50000, K, R, t, seed=53),
        "small": bench_candidates(1500, K, R, t, seed=54),
    }
    want = {k: oracle_scene.score_batch(c, ref, 0.7, 5, nthreads=16) for k, (c, ref) in batches.items()}
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    with pkg.MvsContext(rgb, K, R, t, device=0) as cx:
        overflow = {}
        for j, kind in enumerate(["skewed", "dense", "sparse", "small", "dense", "skewed", "sparse"]):
            c, ref = batches[kind]
            n = len(ref)
            tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
            xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
            rec = torch.full((n, 2), -1, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            before = cx.scorer_stats()
            s = streams[j % 2]
            cx.score_device_rec(tc, tr, xy, rec, 0.7, 5, stream=s.cuda_stream)
            s.synchronize()
            after = cx.scorer_stats()
            oxy, omask, ocount, oavg = want[kind]
            m, cnt = _outputs(rec)
            assert np.array_equal(m, omask[:, 0]) and np.array_equal(cnt, ocount), (j, kind)
            assert np.allclose(rec.cpu().numpy()[:, 1].view(np.float64), oavg, rtol=0, atol=1e-12), (j, kind)
            assert np.array_equal(xy.cpu().numpy(), oxy), (j, kind)
            overflow.setdefault(kind, []).append(after["overflow"] - before["overflow"])
        assert all(v > 0 for v in overflow["skewed"]) and overflow["skewed"][0] == overflow["skewed"][1]
        assert overflow["dense"] == [0, 0] and overflow["sparse"] == [0, 0] and overflow["small"] == [0]

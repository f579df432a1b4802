"""Entry points and configurations beyond the core parity tests (HIP path
against the oracle / the reference's golden vectors):

* MyPatch.photo_consistenecy_test, the per-candidate drop-in (MVS2.py:62-77),
  on the reference's own 300 photo-test cases;
* mvs_expand_candidates (MVS2.py:329-369) against the oracle, on the direct
  (< 2048 jobs) and the tiled (>= 2048) path;
* 47 views at 640x480 (BASELINE config 3's view count, V % 16 != 0) at the
  bench's candidate distribution, through a 2,000-pop stage and through the
  reference's full 100,000-pop expansion (oracle fixture);
* images wider than 2048 pixels;
* device calls on a caller's stream followed by host calls on the context's
  stream (the context's scratch is ordered across streams);
* avg_ncc_score in the reference's own arithmetic (mvs_exact_avg), and the
  opt-in filter_out_outlier mode (MVS2.py:132-158, disabled at MVS2.py:281)
  against the reference run with the filter enabled.
"""
import numpy as np
import pytest

from conftest import bench_candidates

pytestmark = pytest.mark.gpu

AVG_TOL = 1e-12


@pytest.fixture(scope="module")
def ctx(pkg, dino):
    import torch
    assert torch.cuda.is_available(), "GPU test without a GPU"
    rgb, K, R, t = dino
    c = pkg.MvsContext(rgb, K, R, t, device=0)
    yield c
    c.close()


def test_mypatch_dropin_golden(pkg, dino, func_golden):
    """The reference's per-candidate call (MyPatch.photo_consistenecy_test,
    MVS2.py:62-77): V list (views in increasing order, each with the
    projection into the reference view) and avg_ncc_score, on the 300 photo
    tests recorded from the reference itself."""
    import importlib
    mvs2 = importlib.import_module(pkg.__name__ + ".MVS2")
    rgb, K, R, t = dino
    imgs = [rgb[v] for v in range(len(rgb))]
    par_K = {v: K[v] for v in range(len(K))}
    par_r = {v: R[v] for v in range(len(R))}
    par_t = {v: t[v].reshape(3, 1) for v in range(len(t))}
    f = func_golden
    for k in range(len(f["pt_R"])):
        p = mvs2.MyPatch(f["pt_c"][k], None, int(f["pt_R"][k]), [], None, None)
        V = p.photo_consistenecy_test(imgs, par_K, par_r, par_t, float(f["pt_thr"][k]))
        m = int(f["pt_mask"][k, 0])
        views = [b for b in range(64) if (m >> b) & 1]
        assert [e[0] for e in V] == views, k
        assert len(V) == int(f["pt_count"][k])
        for e in V:
            assert e[1] == f["pt_xy"][k, 0] and e[2] == f["pt_xy"][k, 1]
        assert p.avg_ncc_score == f["pt_avg"][k], k   # bit-exact (mvs_exact_avg)
    mvs2.clear_context_cache()


def test_exact_avg_bit_exact(ctx, func_golden):
    """mvs_exact_avg reproduces the reference's avg_ncc_score (MVS2.py:73-76:
    numpy-order ctNcc of every passing view, summed in view order, / |V|) bit
    for bit on its 300 recorded photo tests; mvs_score's own avg within 1e-12."""
    f = func_golden
    for thr in np.unique(f["pt_thr"]):
        sel = f["pt_thr"] == thr
        xy, mask, count, avg = ctx.score(f["pt_c"][sel], f["pt_R"][sel], float(thr), 5)
        ex = ctx.exact_avg(f["pt_R"][sel], xy, mask, 5)
        assert np.array_equal(ex, f["pt_avg"][sel])
        np.testing.assert_allclose(avg, f["pt_avg"][sel], rtol=0, atol=AVG_TOL)


@pytest.mark.parametrize("cap", [200, 1000])
def test_stage_filter_outliers_vs_reference(ctx, seeds, cap):
    """filter_out_outlier enabled (opt-in): the reference itself run with the
    filter before reconstruct_from_Q at 200- and 1000-pop caps
    (tests/golden/gen_golden.py --filter-stage) -- same rows, same number of
    "remove a outlier" lines."""
    import os
    from conftest import GOLDEN
    p = os.path.join(GOLDEN, f"stage_filter_cap{cap}.npz")
    g = dict(np.load(p))
    assert int(g["pops"]) == cap
    ini, allp, st = ctx.stage(seeds["track_off"], seeds["obs_view"], seeds["obs_xy"],
                              cell_size=2, scale=10.0, wid=5, max_pops=cap, filter_outliers=True)
    assert np.array_equal(ini, g["initial_patches"])
    assert np.array_equal(allp, g["all_patches"])
    assert st["outlier_lines"] == int(g["removed_lines"])


def test_stage_filter_outliers_full_run(ctx, seeds):
    """At the reference's 100k pops the filter removes nothing and the rows are
    the unfiltered run's: an accepted patch has |V| >= 2 views each with ncc >
    MIN_NCC >= 0.4, so |V|·avg > 0.8 while a cell's threshold, the mean of
    1 - avg, is < 0.6 (MVS2.py:142-148)."""
    ini0, all0, st0 = ctx.stage(seeds["track_off"], seeds["obs_view"], seeds["obs_xy"],
                                cell_size=2, scale=10.0, wid=5, max_pops=100000)
    ini, allp, st = ctx.stage(seeds["track_off"], seeds["obs_view"], seeds["obs_xy"],
                              cell_size=2, scale=10.0, wid=5, max_pops=100000, filter_outliers=True)
    assert st["outliers_removed"] == 0 and st["outlier_lines"] == 0
    assert st["accepts"] == st0["accepts"]
    assert np.array_equal(ini, ini0) and np.array_equal(allp, all0)
    ctx.set_stage_options(False)


def test_mypatch_context_follows_image_edits(pkg, dino):
    """The cached scene context sees in-place edits of the images (sampled
    content fingerprint) and replaced arrays."""
    import importlib
    mvs2 = importlib.import_module(pkg.__name__ + ".MVS2")
    rgb, K, R, t = dino
    imgs = [rgb[v].copy() for v in range(len(rgb))]
    par = ({v: K[v] for v in range(48)}, {v: R[v] for v in range(48)},
           {v: t[v].reshape(3, 1) for v in range(48)})
    c1 = mvs2.scene_context(imgs, *par)
    assert mvs2.scene_context(imgs, *par) is c1
    imgs[3][0, :, :] = 7                       # row 0 is sampled
    c2 = mvs2.scene_context(imgs, *par)
    assert c2 is not c1
    imgs[5] = imgs[5].copy()                    # a new array object
    assert mvs2.scene_context(imgs, *par) is not c2
    mvs2.clear_context_cache()


def _parents(K, R, t, n, seed):
    """Parent patches on the object's depth range: centre, normal toward the
    reference camera, projection into the reference view (MVS2.py:238-247)."""
    from oracle import oracle as orc
    c, ref = bench_candidates(n, K, R, t, seed=seed)
    pn = np.empty_like(c)
    pxy = np.empty((n, 2))
    for k in range(n):
        O = -(R[ref[k]].T @ t[ref[k]].ravel())
        d = O - c[k]
        pn[k] = d / np.linalg.norm(d)
        pxy[k] = orc.project(K[ref[k]], orc.rodrigues_roundtrip(R[ref[k]]), t[ref[k]].ravel(), c[k])
    return c, pn, pxy, ref


@pytest.mark.parametrize("n_jobs", [700, 4096])
def test_expand_candidates_vs_oracle(ctx, oracle_scene, dino, n_jobs):
    """mvs_expand_candidates: every output of every job bit-exact against the
    oracle's restatement of MVS2.py:329-369 (direct path below 2,048 jobs,
    geometry + tiled photo test + accept above)."""
    rgb, K, R, t = dino
    rng = np.random.default_rng(n_jobs)
    pc, pn, pxy, _ = _parents(K, R, t, 400, seed=n_jobs)
    jp = rng.integers(0, len(pc), n_jobs).astype(np.int32)
    jv = rng.integers(0, 48, n_jobs).astype(np.int32)
    jd = rng.choice(np.array([-1, 1], np.int32), n_jobs)
    got = ctx.expand_candidates(pc, pn, pxy, jp, jv, jd, cell_size=2, scale=10.0, wid=5, min_ncc=0.7)
    exp = oracle_scene.expand_candidates(pc, pn, pxy, jp, jv, jd, cell_size=2, scale=10.0, wid=5, thr=0.7)
    for name, g, e in zip(("X", "nX", "color", "xy", "mask", "count", "accept"), got, exp):
        assert np.array_equal(g, e), name
    assert exp[5].sum() > 0


@pytest.fixture(scope="module")
def dino47(dino):
    rgb, K, R, t = dino
    return rgb[:47].copy(), K[:47].copy(), R[:47].copy(), t[:47].copy()


def test_view_count_47_bench_distribution(pkg, orc, dino47):
    """47 views of 640x480 (BASELINE config 3's view count; the last 16-view
    block of the matrix-core scorer is padded): 2^18 candidates of the bench's
    distribution bit-exact against the oracle."""
    import os
    rgb, K, R, t = dino47
    c, ref = pkg.synthetic.candidates(1 << 18, K, R, t, seed=47)
    with pkg.MvsContext(rgb, K, R, t) as cx:
        got = cx.score(c, ref, 0.7, 5)
    exp = orc.Scene(rgb, K, R, t).score_batch(c, ref, 0.7, 5, nthreads=min(os.cpu_count() or 1, 16))
    for g, e in zip(got[:3], exp[:3]):
        assert np.array_equal(g, e)
    np.testing.assert_allclose(got[3], exp[3], rtol=0, atol=AVG_TOL)
    assert got[2].sum() > 0


def test_view_count_47_stage(pkg, orc, dino47, seeds):
    """The 47-view scene through a 2,000-pop stage (seeds restricted to
    tracks inside views 0-46), bit-exact against the oracle stage."""
    from make_seeds import subset_seeds
    rgb, K, R, t = dino47
    args = subset_seeds(seeds, 47)
    with pkg.MvsContext(rgb, K, R, t) as cx:
        ini, allp, st = cx.stage(*args, cell_size=2, scale=10.0, wid=5, max_pops=2000)
    oini, oall, ost = orc.Scene(rgb, K, R, t).mvs_stage(*args, scale=10.0, max_pops=2000)
    assert st["pops"] == ost["pops"] and st["tests"] == ost["tests"]
    assert np.array_equal(ini, oini) and np.array_equal(allp, oall)
    assert len(allp) > 1000


def test_view_count_47_full_run_vs_oracle_fixture(pkg, dino47, seeds):
    """BASELINE config 3 at full length: 47 views (templeRing is absent, so the
    dinoRing subset of views 0-46 stands in) through the
    reference's whole 100,000-pop expansion (MVS2.py:321).  Every accepted
    patch, in order, against the oracle's full run
    (tests/golden/gen_oracle_full.py 100000 47: counts + sha256 of both row
    sets)."""
    import hashlib
    import json
    import os
    from conftest import GOLDEN
    from make_seeds import subset_seeds
    j = json.load(open(os.path.join(GOLDEN, "stage_oracle_v47_cap100000.json")))
    rgb, K, R, t = dino47
    with pkg.MvsContext(rgb, K, R, t) as cx:
        ini, allp, st = cx.stage(*subset_seeds(seeds, 47), cell_size=2, scale=10.0, wid=5,
                                 max_pops=100000)
    for k in ("pops", "tests", "queue_left"):
        assert st[k] == j["stats"][k], k
    assert len(ini) == j["n_initial"] and len(allp) == j["n_all"]
    assert hashlib.sha256(np.ascontiguousarray(ini, "<f8").tobytes()).hexdigest() == j["sha256_initial"]
    assert hashlib.sha256(np.ascontiguousarray(allp, "<f8").tobytes()).hexdigest() == j["sha256_all"]


def test_wide_image(pkg, orc):
    """W = 2100 (> 2048): tile coordinates are stored relative to the tile,
    so any width/height works; every output against the oracle."""
    H, W, V = 64, 2100, 6
    rgb, K, R, t = pkg.synthetic.ring_scene(V=V, H=H, W=W, seed=3)
    rgb = ((rgb.astype(np.uint16) + np.roll(rgb, 1, axis=0)) // 2).astype(np.uint8)
    c, ref = pkg.synthetic.candidates(6000, K, R, t, W=W, H=H, seed=3)
    with pkg.MvsContext(rgb, K, R, t) as cx:
        got = cx.score(c, ref, 0.2, 5)
    exp = orc.Scene(rgb, K, R, t).score_batch(c, ref, 0.2, 5)
    for g, e in zip(got[:3], exp[:3]):
        assert np.array_equal(g, e)
    assert (got[2] > 0).any() and (np.asarray(got[0])[:, 0] > 2048).any()


def test_device_call_on_other_stream_then_host_call(ctx, oracle_scene, dino):
    """A scoring call on a caller's stream, then at once a host-pointer call on
    the context's own stream: the second waits for the first's use of the
    shared scratch, both results are right."""
    import torch
    rgb, K, R, t = dino
    c1, r1 = bench_candidates(1 << 16, K, R, t, seed=31)
    c2, r2 = bench_candidates(5000, K, R, t, seed=32)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        tc = torch.from_numpy(c1).to(dev)
        tr = torch.from_numpy(r1).to(dev)
        xy = torch.empty((len(r1), 2), dtype=torch.float64, device=dev)
        mask = torch.empty((len(r1), 1), dtype=torch.int64, device=dev)
        count = torch.empty(len(r1), dtype=torch.int32, device=dev)
        avg = torch.empty(len(r1), dtype=torch.float64, device=dev)
    ctx.score_device(tc, tr, xy, mask, count, avg, 0.7, 5, stream=s.cuda_stream)
    got2 = ctx.score(c2, r2, 0.7, 5)                     # context stream, right away
    s.synchronize()
    exp1 = oracle_scene.score_batch(c1, r1, 0.7, 5, nthreads=8)
    exp2 = oracle_scene.score_batch(c2, r2, 0.7, 5, nthreads=8)
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), exp1[1])
    assert np.array_equal(count.cpu().numpy(), exp1[2])
    assert np.array_equal(got2[1], exp2[1]) and np.array_equal(got2[2], exp2[2])


def test_timed_kernel_name(ctx, dino):
    rgb, K, R, t = dino
    c, ref = bench_candidates(4096, K, R, t, seed=1)
    ctx.kernel_timing(True)
    ctx.score(c, ref, 0.7, 5)
    ms, k = ctx.kernel_time()
    ctx.kernel_timing(False)
    assert k == 1 and ms > 0 and ctx.timed_kernel() == "k_score_tab"


def test_pack_accepted_vs_reference_and_time(pkg, ctx, dino):
    """mvs_pack_accepted (the multi-GPU exchange's device pack, no host sync)
    against parallel.pack_accepted_reference on the bench's 2^20 sweep: the
    same header and the same rows once ordered by index (the pack keeps each
    8,192-candidate chunk in index order, the chunks in reservation order) --
    with the accepted 3D points (40-B rows, the bench's exchange) and without
    (16-B rows) -- including a capacity below the accepted count (cap distinct
    accepted rows, the true count in the header) and an empty slice.  The
    pack's device time per call is printed and bounded (15 us per 2^20 sweep,
    launch gaps included)."""
    import importlib
    import torch
    par = importlib.import_module(pkg.__name__ + ".parallel")
    rgb, K, R, t = dino
    n = 1 << 20
    c, ref = bench_candidates(n, K, R, t, seed=0)
    dev = torch.device("cuda:0")
    tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    mask = torch.empty((n, 1), dtype=torch.int64, device=dev)
    count = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.score_device(tc, tr, xy, mask, count, None, 0.7, 5)
    torch.cuda.synchronize()
    acc = int((count >= 3).sum())
    assert acc > 1000
    for pts in (False, True):
        w = par.points_width(1, pts)
        exp = torch.full((acc + 1, w), -9, dtype=torch.int64)
        for cap, off in ((acc + 300, 5 << 20), (acc // 3, 0)):
            out = torch.full((cap + 1, w), -9, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            ctx.pack_accepted(off, count, mask, 3, out, c=tc if pts else None)   # the library's stream
            torch.cuda.synchronize()
            par.pack_accepted_reference(off, count.cpu(), mask.cpu(), 3, exp, torch.from_numpy(c) if pts else None)
            got = out.cpu()
            k = min(acc, cap)
            assert got[0].tolist() == [acc, n] + [0] * (w - 2)
            rows = par.sort_rows(got[1:1 + k])
            if cap >= acc:
                assert torch.equal(rows, exp[1:1 + acc])
                assert (got[1 + acc:] == -9).all()
            else:   # cap rows, each one of the accepted rows, none twice
                pos = torch.searchsorted(exp[1:, 0].contiguous(), rows[:, 0].contiguous())
                assert torch.equal(rows, exp[1:][pos]) and int(torch.unique(rows[:, 0]).numel()) == k
            if pts:   # the rows carry the candidates' own centres, bit for bit
                idx = rows[:, 0].numpy() - off
                assert np.array_equal(rows[:, 2:5].contiguous().view(torch.float64).numpy(), c[idx])
    empty = torch.full((4, 2), -9, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ctx.pack_accepted(0, count[:0], mask[:0], 3, empty)
    torch.cuda.synchronize()
    assert empty[0].cpu().tolist() == [0, 0]
    # a stream of our own: torch's default stream is handle 0, which the
    # C-ABI reads as the context's own stream (the events would not bracket it)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    for pts in (False, True):
        out = torch.empty((acc + 300 + 1, par.points_width(1, pts)), dtype=torch.int64, device=dev)
        cc = tc if pts else None
        for _ in range(3):
            ctx.pack_accepted(0, count, mask, 3, out, stream=s.cuda_stream, c=cc)
        # the packs queue behind scoring work (~1 ms of it), so that the events
        # time the device and not the host's submission rate (~15 us per call)
        for _ in range(10):
            ctx.score_device(tc, tr, xy, mask, count, None, 0.7, 5, stream=s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            ctx.pack_accepted(0, count, mask, 3, out, stream=s.cuda_stream, c=cc)
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"pack_accepted ({'40' if pts else '16'}-B rows): {us:.1f} us per 2^20 sweep ({acc} accepted rows)")
        assert int(out[0, 0]) == acc
        # events around back-to-back launches include the inter-kernel gaps;
        # the kernel's own time is in the rocprof summaries (profiles/r06/)
        assert us <= 15.0


@pytest.mark.parametrize("n", [1, 8191, 8193, 200_001, 5_000_001])
def test_pack_accepted_sizes(pkg, ctx, n):
    """The pack over 8,192-candidate chunks (one workgroup each, one row
    reservation each): a single partial chunk, a chunk boundary, 25 chunks,
    and more chunks (611 at 5M) than workgroups resident at once; synthetic
    counts/masks against the torch reference, three calls in a row on two
    streams with an empty slice between them (the counter and the ticket
    must come back to zero after every call)."""
    import importlib
    import torch
    par = importlib.import_module(pkg.__name__ + ".parallel")
    g = torch.Generator().manual_seed(n)
    count = torch.randint(0, 8, (n,), generator=g, dtype=torch.int32)
    mask = torch.randint(-2**62, 2**62, (n, 1), generator=g, dtype=torch.int64)
    acc = int((count >= 3).sum())
    exp = torch.full((acc + 2, 2), -9, dtype=torch.int64)
    par.pack_accepted_reference(7, count, mask, 3, exp)
    dc, dm = count.cuda(), mask.cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for k in range(3):
        out = torch.full((acc + 2, 2), -9, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        s = streams[k & 1]
        ctx.pack_accepted(7, dc, dm, 3, out, stream=s.cuda_stream)
        if k == 1:
            e = torch.full((2, 2), -9, dtype=torch.int64, device="cuda")
            ctx.pack_accepted(0, dc[:0], dm[:0], 3, e, stream=streams[0].cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu()
        assert got[0].tolist() == [acc, n]
        assert torch.equal(par.sort_rows(got[1:1 + acc]), exp[1:1 + acc])
        assert got[1 + acc].tolist() == [-9, -9]
        if k == 1:
            assert e[0].cpu().tolist() == [0, 0]


def test_score_records_vs_arrays_and_pack(pkg, ctx, dino, orc):
    """mvs_score_device_rec (one [mask, avg] record per candidate, |V| by
    popcount) gives the three-array outputs bit for bit -- tiled scorer (the
    bench's 2^20 sweep, and the oracle on its first 20k candidates) and direct
    path (a small batch) -- and the pack reads the records (d_count NULL) into
    the same exchange rows as from the arrays."""
    import importlib
    import torch
    par = importlib.import_module(pkg.__name__ + ".parallel")
    rgb, K, R, t = dino
    dev = torch.device("cuda:0")
    for n in (1 << 20, 1500):
        c, ref = bench_candidates(n, K, R, t, seed=11)
        tc, tr = torch.from_numpy(c).to(dev), torch.from_numpy(ref).to(dev)
        xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
        mask = torch.empty((n, 1), dtype=torch.int64, device=dev)
        count = torch.empty(n, dtype=torch.int32, device=dev)
        avg = torch.empty(n, dtype=torch.float64, device=dev)
        rec = torch.full((n, 2), -5, dtype=torch.int64, device=dev)
        xy2 = torch.empty_like(xy)
        torch.cuda.synchronize()
        ctx.score_device(tc, tr, xy, mask, count, avg, 0.7, 5)
        torch.cuda.synchronize()
        ctx.score_device_rec(tc, tr, xy2, rec, 0.7, 5)
        torch.cuda.synchronize()
        r = rec.cpu().numpy()
        m = mask.cpu().numpy()
        assert np.array_equal(r[:, 0], m[:, 0]) and np.array_equal(xy.cpu().numpy(), xy2.cpu().numpy())
        assert np.array_equal(np.bitwise_count(r[:, 0].view(np.uint64)).astype(np.int32), count.cpu().numpy())
        assert np.array_equal(r[:, 1].view(np.float64), avg.cpu().numpy())
        k = min(n, 20000)
        oxy, omask, ocount, oavg = orc.Scene(rgb, K, R, t).score_batch(c[:k], ref[:k], 0.7, 5, nthreads=8)
        assert np.array_equal(r[:k, 0].view(np.uint64), omask[:, 0])
        assert np.allclose(r[:k, 1].view(np.float64), oavg, rtol=0, atol=AVG_TOL)
        acc = int((count >= 3).sum())
        w = par.points_width(1)
        o1 = torch.full((acc + 5, w), -9, dtype=torch.int64, device=dev)
        o2 = torch.full((acc + 5, w), -9, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        ctx.pack_accepted(3, count, mask, 3, o1, c=tc)
        ctx.pack_accepted(3, None, rec, 3, o2, c=tc)
        torch.cuda.synchronize()
        r1, r2 = o1.cpu(), o2.cpu()
        assert int(r1[0, 0]) == acc and torch.equal(r1[0], r2[0])
        assert torch.equal(par.sort_rows(r1[1:1 + acc]), par.sort_rows(r2[1:1 + acc]))
        exp = torch.full((acc + 5, w), -9, dtype=torch.int64)
        par.pack_accepted_reference(3, None, rec.cpu(), 3, exp, torch.from_numpy(c))
        assert torch.equal(r2[0], exp[0]) and torch.equal(par.sort_rows(r2[1:1 + acc]), exp[1:1 + acc])


def test_skewed_batch_overflow_cost(pkg, ctx, dino, orc):
    """A skewed sweep: 2^18 candidates crowded onto two pixel tiles,
    so that most of them overflow the tile buckets (cap = 16x the mean load)
    into the direct path's list.  Outputs stay exact (a 4,000-candidate sample
    against the oracle) and the whole call stays bounded: the direct path's
    grid grows with the batch (up to 256 workgroups)."""
    import time
    import torch
    rgb, K, R, t = dino
    rng = np.random.default_rng(13)
    n = 1 << 18
    ref = rng.integers(0, 48, n).astype(np.int32)
    x = np.where(rng.random(n) < 0.5, 300.0, 333.0) + rng.random(n) * 15.9
    y = 200 + rng.random(n) * 7.9
    z = rng.uniform(0.6, 0.72, n)
    Kinv = np.linalg.inv(K)
    ray = np.einsum("nij,nj->ni", Kinv[ref], np.stack([x, y, np.ones(n)], 1))
    c = np.einsum("nji,nj->ni", R[ref], z[:, None] * ray - t[ref].reshape(n, 3))
    dev = torch.device("cuda:0")
    tc, tr = torch.from_numpy(np.ascontiguousarray(c)).to(dev), torch.from_numpy(ref).to(dev)
    xy = torch.empty((n, 2), dtype=torch.float64, device=dev)
    mask = torch.empty((n, 1), dtype=torch.int64, device=dev)
    count = torch.empty(n, dtype=torch.int32, device=dev)
    avg = torch.empty(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.score_device(tc, tr, xy, mask, count, avg, 0.7, 5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.score_device(tc, tr, xy, mask, count, avg, 0.7, 5)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"skewed 2^18 batch (2 tiles): {ms:.2f} ms")
    k = rng.choice(n, 4000, replace=False)
    oxy, omask, ocount, oavg = orc.Scene(rgb, K, R, t).score_batch(c[k], ref[k], 0.7, 5, nthreads=8)
    assert np.array_equal(mask.cpu().numpy()[k].view(np.uint64), omask)
    assert np.array_equal(count.cpu().numpy()[k], ocount)
    np.testing.assert_allclose(avg.cpu().numpy()[k], oavg, rtol=0, atol=AVG_TOL)
    assert ms < 20.0


def test_in_kernel_moments_path(pkg, dino, orc):
    """The scorer without the per-scene window-moment tables (k_score_mma, the
    path for scenes whose tables would not fit; MVS_SCORE_KERNEL=mma) against
    the tables path and the oracle on the bench's candidates."""
    import os
    rgb, K, R, t = dino
    c, ref = bench_candidates(1 << 17, K, R, t, seed=4)
    os.environ["MVS_SCORE_KERNEL"] = "mma"
    try:
        cm = pkg.MvsContext(rgb, K, R, t, device=0)
    finally:
        del os.environ["MVS_SCORE_KERNEL"]
    try:
        cm.kernel_timing(True)
        got = cm.score(c, ref, 0.7, 5)
        cm.kernel_timing(False)
        assert cm.timed_kernel() == "k_score_mma"
    finally:
        cm.close()
    with pkg.MvsContext(rgb, K, R, t, device=0) as ct:
        tab = ct.score(c, ref, 0.7, 5)
    for g, e in zip(got[:3], tab[:3]):
        assert np.array_equal(g, e)
    np.testing.assert_allclose(got[3], tab[3], rtol=0, atol=AVG_TOL)
    k = 5000
    oxy, omask, ocount, oavg = orc.Scene(rgb, K, R, t).score_batch(c[:k], ref[:k], 0.7, 5, nthreads=8)
    assert np.array_equal(got[1][:k], omask) and np.array_equal(got[2][:k], ocount)

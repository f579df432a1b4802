"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own
code (MVS2.py, HarrisFeatures.py, utils.py at /root/reference) in this
container, with the OpenCV / pyntcloud stand-ins of tests/golden/standins/.

Run here only (the reference never travels to the GPU box):
    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/gen_golden.py [--stage CAP ...]

Outputs (all data, no reference source):
  seeds_dino.npz        synthetic 2-view SfM tracks (make_seeds.py recipe)
  func_golden.npz       getDescFeatures+ctNcc pairs, projectPoint, photo tests,
                        ray_plane_intersection / is_patch_neighbor samples
  stage_cap{N}.npz      DensePointsWithMVS2 outputs (initial_patches,
                        all_patches rows) on dinoRing + seeds, queue capped at N pops
  stage_filter_cap{N}.npz  the same with the reference's filter_out_outlier
                        (MVS2.py:132-158) enabled where MVS2.py:281 has it commented
                        out: reconstruct_from_Q (called right after, MVS2.py:285) is
                        wrapped to run the filter first; also the number of
                        "remove a outlier" lines it printed
  filter_crafted.npz    filter_out_outlier on crafted patch sets (stub patches
                        with random avg / normals / V lists) where it removes
                        patches or raises ZeroDivisionError
"""
import argparse
import contextlib
import io
import os
import queue as _queue
import sys
import time

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "standins"))
sys.path.insert(1, REF)
sys.path.insert(2, REPO)
sys.path.insert(3, HERE)

import numpy as np  # noqa: E402

from make_seeds import load_dino, make_seeds  # noqa: E402
from oracle import oracle as orc  # noqa: E402

DATA = os.path.join(REPO, "data", "dinoRing")
PAR = os.path.join(DATA, "dinoR_par.txt")


class Args:
    par_path = PAR
    scale = 10.0
    cell_size = 2
    desc_wid = 5
    debug = False


class Track:
    def __init__(self, obs):
        self.point2d_list = obs


class SeedSet:
    """Stands in for GlobalSet: getInfo() -> (n_obs, n_pts, tracks) (GlobalSet.py:36-50)."""

    def __init__(self, tracks):
        self.tracks = tracks

    def getInfo(self):
        return 0, len(self.tracks), self.tracks


def seeds_to_tracks(seeds):
    off, view, xy = seeds["track_off"], seeds["obs_view"], seeds["obs_xy"].astype(np.float32)
    tracks = []
    for k in range(len(off) - 1):
        tracks.append(Track([(int(view[o]), xy[o, 0], xy[o, 1]) for o in range(off[k], off[k + 1])]))
    return tracks


def import_reference():
    import MVS2  # the reference module, unmodified
    return MVS2


def func_golden(MVS2, imgs, K, Rm, t, rng):
    import HarrisFeatures
    import utils
    out = {}
    V = len(imgs)
    H, W = imgs[0].shape[:2]
    gray = [np.asarray(sys.modules["cv2"].cvtColor(im, 6)) for im in imgs]
    # --- window + ctNcc pairs (HarrisFeatures.py:116-133, MVS2.py:39-43) ---
    for wid in (5, 3):
        A, B, S = [], [], []
        n = 3000
        while len(S) < n:
            v1, v2 = rng.integers(0, V, 2)
            y = rng.uniform(wid, H - wid - 1)
            x = rng.uniform(wid + 1, W - wid - 1)
            if len(S) % 3 == 0:   # near the object: mostly textured windows
                y = rng.uniform(120, 400)
                x = rng.uniform(150, 500)
            da = HarrisFeatures.getDescFeatures(imgs[v1], np.array([[y, x]]), wid=wid)[0]
            db = HarrisFeatures.getDescFeatures(imgs[v2], np.array([[y, x]]), wid=wid)[0]
            if da is None or db is None:
                continue
            with np.errstate(all="ignore"):
                s = MVS2.ctNcc(da, db)
            A.append(da); B.append(db); S.append(s)
        # synthetic windows: random, near-constant, constant, near-threshold pairs
        npx = (2 * wid + 1) ** 2
        for k in range(600):
            kind = k % 4
            if kind == 0:
                a = rng.integers(0, 256, npx, dtype=np.uint8); b = rng.integers(0, 256, npx, dtype=np.uint8)
            elif kind == 1:
                a = np.full(npx, rng.integers(0, 256), np.uint8); b = rng.integers(0, 256, npx, dtype=np.uint8)
            elif kind == 2:
                a = rng.integers(0, 256, npx, dtype=np.uint8)
                b = np.clip(a.astype(int) + rng.integers(-60, 61, npx), 0, 255).astype(np.uint8)
            else:
                a = np.clip(100 + rng.integers(-2, 3, npx), 0, 255).astype(np.uint8)
                b = np.clip(a.astype(int) + rng.integers(-1, 2, npx), 0, 255).astype(np.uint8)
            with np.errstate(all="ignore"):
                s = MVS2.ctNcc(a, b)
            A.append(a); B.append(b); S.append(s)
        out[f"ncc_a_w{wid}"] = np.stack(A)
        out[f"ncc_b_w{wid}"] = np.stack(B)
        out[f"ncc_s_w{wid}"] = np.array(S, np.float64)
    # --- window validity edge cases (HarrisFeatures.py:128) ---
    cases = []
    for y in (4.9, 5.0, 5.5, H - 7.0, H - 6.5, H - 6.0, -0.5, -1.0):
        for x in (5.9, 6.0, 6.5, W - 7.0, W - 6.5, W - 6.0, -0.2):
            d = HarrisFeatures.getDescFeatures(imgs[0], np.array([[y, x]]), wid=5)[0]
            cases.append((y, x, d is not None))
    out["desc_edge"] = np.array(cases, np.float64)
    # --- projectPoint (utils.py:241-244) ---
    P, C, R_ = [], [], []
    for k in range(500):
        v = int(rng.integers(0, V))
        c = rng.uniform([-0.03, 0.01, -0.03], [0.06, 0.12, 0.06])
        P.append(utils.projectPoint(c, Rm[v], t[v], K[v])); C.append(c); R_.append(v)
    out["proj_c"] = np.array(C); out["proj_v"] = np.array(R_, np.int32); out["proj_xy"] = np.array(P)
    # --- photo_consistenecy_test (MVS2.py:62-77) on bench-distribution candidates ---
    cs, rs, thrs, Vs, avgs, xys = [], [], [], [], [], []
    Kinv = [np.linalg.inv(k) for k in K]
    for k in range(300):
        v = int(rng.integers(0, V))
        x = rng.uniform(6, 633) if k % 2 else rng.uniform(150, 500)
        y = rng.uniform(5, 473) if k % 2 else rng.uniform(100, 420)
        z = rng.uniform(0.60, 0.72)
        ray = Kinv[v] @ np.array([x, y, 1.0])
        c = Rm[v].T @ (z * ray - t[v].ravel())
        thr = 0.7 if k % 3 else 0.4
        p = MVS2.MyPatch(c, None, v, None, None, None)
        with np.errstate(all="ignore"):
            Vl = p.photo_consistenecy_test(imgs, K, Rm, t, MIN_NCC=thr)
        cs.append(c); rs.append(v); thrs.append(thr)
        Vs.append([e[0] for e in Vl]); avgs.append(p.avg_ncc_score)
        xys.append(utils.projectPoint(c, Rm[v], t[v], K[v]))
    out["pt_c"] = np.array(cs); out["pt_R"] = np.array(rs, np.int32); out["pt_thr"] = np.array(thrs)
    words = (V + 63) // 64
    mask = np.zeros((len(Vs), words), np.uint64)
    for i, vl in enumerate(Vs):
        for e in vl:
            mask[i, e // 64] |= np.uint64(1) << np.uint64(e % 64)
    out["pt_mask"] = mask
    out["pt_count"] = np.array([len(v) for v in Vs], np.int32)
    out["pt_avg"] = np.array(avgs, np.float64)
    out["pt_xy"] = np.array(xys)
    # --- ray_plane_intersection / is_patch_neighbor (MVS2.py:298-306) ---
    rp = []
    for k in range(500):
        o = rng.normal(size=3); d = rng.normal(size=3); d /= np.linalg.norm(d)
        pc = rng.normal(size=3); pn = rng.normal(size=3); pn /= np.linalg.norm(pn)
        X = MVS2.ray_plane_intersection(o, d, pc, pn)
        a = MVS2.MyPatch(pc, pn, 0, None, None, None)
        xn = rng.normal(size=3); xn /= np.linalg.norm(xn)
        b = MVS2.MyPatch(X, xn, 0, None, None, None)
        nb = MVS2.is_patch_neighbor(a, b, threshold=0.1)
        rp.append(np.concatenate([o, d, pc, pn, X, xn, [float(nb)]]))
    out["rayplane"] = np.array(rp)
    return out


def stage_golden(MVS2, imgs, tracks, cap, with_filter=False):
    import pyntcloud

    class CappedQueue(_queue.Queue):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.gets = 0

        def get(self, *a, **k):
            self.gets += 1
            return super().get(*a, **k)

        def empty(self):
            return self.gets >= cap or super().empty()

    orig_queue = MVS2.queue.Queue
    MVS2.queue.Queue = CappedQueue
    orig_reconstruct = MVS2.CellTable.reconstruct_from_Q
    if with_filter:
        def reconstruct_after_filter(self):
            self.filter_out_outlier()
            return orig_reconstruct(self)
        MVS2.CellTable.reconstruct_from_Q = reconstruct_after_filter
    pyntcloud.written.clear()
    t0 = time.time()
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf), np.errstate(all="ignore"):
            MVS2.DensePointsWithMVS2(imgs, SeedSet(tracks), Args())
    finally:
        # restored, so that a second run in this process does not subclass this
        # run's queue (its gets would then count twice)
        MVS2.queue.Queue = orig_queue
        MVS2.CellTable.reconstruct_from_Q = orig_reconstruct
    dt = time.time() - t0
    ntests = buf.getvalue().count("iteration:")
    out = {"initial_patches": pyntcloud.written["initial_patches.ply"],
           "all_patches": pyntcloud.written["all_patches.ply"],
           "cap": np.int64(cap), "ref_seconds": np.float64(dt), "pops": np.int64(ntests)}
    if with_filter:
        out["removed_lines"] = np.int64(buf.getvalue().count("remove a outlier"))
    return out


def filter_crafted_golden(MVS2, n_cases=60, seed=2024):
    """filter_out_outlier (MVS2.py:132-158) on crafted patch sets, where it
    does remove patches (with the stage's own parameters it provably cannot,
    DESIGN 4.3): stub MyPatch objects (MVS2.py:45-57) with random centres,
    normals, avg_ncc_score and V lists (every entry at the patch's own x, y,
    as the photo test produces them, MVS2.py:68/74) are filled into a CellTable
    (MVS2.py:401-403: fill_with_point per V entry), then the reference's
    filter runs and reconstruct_from_Q (MVS2.py:159-173) gives the survivors'
    order.  Per case: the inputs in fill order, the survivor ids in output
    order, the "remove a outlier" line count, and whether the filter raised
    ZeroDivisionError (a filled cell emptied before its visit, MVS2.py:144)."""
    rng = np.random.default_rng(seed)
    H = W = 13                     # cell grid ceil(12/2) = 6 x 6 per view at cell size 2
    cs = 2
    out = {"cs": np.int64(cs), "H": np.int64(H), "W": np.int64(W)}
    for k in range(n_cases):
        V = int(rng.integers(2, 7))
        npatch = int(rng.integers(2, 40))
        ncell = int(rng.integers(1, 5))            # few cells: patches collide in them
        cells = rng.integers(0, 6, (ncell, 2))
        spread = float(rng.choice([0.05, 0.2, 0.5]))
        imgs = [np.zeros((H, W), np.uint8) for _ in range(V)]
        table = MVS2.CellTable(imgs, cell_size=cs)
        pid, pview, pxy, pc, pn, pavg = [], [], [], [], [], []
        patches = []
        for p in range(npatch):
            ci, cj = cells[rng.integers(0, ncell)]
            x = cs * ci + rng.uniform(0, cs - 1e-6)
            y = cs * cj + rng.uniform(0, cs - 1e-6)
            nv = int(rng.integers(1, V + 1))
            views = np.sort(rng.choice(V, nv, replace=False))
            c = rng.normal(0, spread, 3)
            nrm = rng.normal(0, 1, 3)
            nrm /= np.linalg.norm(nrm)
            obj = MVS2.MyPatch(c, nrm, int(views[0]), [[int(v), x, y] for v in views], np.array([p, 0, 0]), None)
            obj.avg_ncc_score = float(rng.uniform(0.05, 0.95))
            patches.append(obj)
            mask = 0
            for v in views:
                mask |= 1 << int(v)
            pid.append(p); pview.append(mask); pxy.append((x, y)); pc.append(c); pn.append(nrm)
            pavg.append(obj.avg_ncc_score)
            for h in obj.V:
                table.fill_with_point(h[0], h[1], h[2], obj)
        buf = io.StringIO()
        divzero = False
        try:
            with contextlib.redirect_stdout(buf):
                table.filter_out_outlier()
        except ZeroDivisionError:
            divzero = True
        lines = buf.getvalue().count("remove a outlier")
        surv = []
        if not divzero:
            pts, cols = table.reconstruct_from_Q()
            surv = [int(col[0]) for col in cols]
        out[f"c{k}_V"] = np.int64(V)
        out[f"c{k}_mask"] = np.array(pview, np.uint64)
        out[f"c{k}_xy"] = np.array(pxy, np.float64)
        out[f"c{k}_c"] = np.array(pc, np.float64)
        out[f"c{k}_n"] = np.array(pn, np.float64)
        out[f"c{k}_avg"] = np.array(pavg, np.float64)
        out[f"c{k}_survivors"] = np.array(surv, np.int64)
        out[f"c{k}_lines"] = np.int64(lines)
        out[f"c{k}_divzero"] = np.bool_(divzero)
    out["n_cases"] = np.int64(n_cases)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--func", action="store_true")
    ap.add_argument("--seeds", action="store_true")
    ap.add_argument("--stage", type=int, nargs="*", default=[])
    ap.add_argument("--filter-stage", type=int, nargs="*", default=[])
    ap.add_argument("--filter-crafted", action="store_true")
    a = ap.parse_args()
    assert os.path.isdir(REF), "the reference is only present in the build container"
    imgs, K, Rm, t = load_dino(DATA)
    if a.seeds or not os.path.exists(os.path.join(HERE, "seeds_dino.npz")):
        seeds = make_seeds(imgs, K, Rm, t)
        np.savez_compressed(os.path.join(HERE, "seeds_dino.npz"), **seeds)
        print("seeds:", len(seeds["track_off"]) - 1, "tracks")
    seeds = dict(np.load(os.path.join(HERE, "seeds_dino.npz")))
    MVS2 = import_reference()
    if a.func:
        rng = np.random.default_rng(12345)
        out = func_golden(MVS2, imgs, K, Rm, t, rng)
        np.savez_compressed(os.path.join(HERE, "func_golden.npz"), **out)
        print("func golden written", {k: v.shape for k, v in out.items()})
    if a.filter_crafted:
        out = filter_crafted_golden(MVS2)
        np.savez_compressed(os.path.join(HERE, "filter_crafted.npz"), **out)
        nrem = sum(int(out[f"c{k}_lines"]) > 0 for k in range(int(out["n_cases"])))
        ndz = sum(bool(out[f"c{k}_divzero"]) for k in range(int(out["n_cases"])))
        print(f"filter_crafted: {int(out['n_cases'])} cases, {nrem} with removals, {ndz} ZeroDivisionError")
    for cap in a.stage:
        out = stage_golden(MVS2, imgs, seeds_to_tracks(seeds), cap)
        np.savez_compressed(os.path.join(HERE, f"stage_cap{cap}.npz"), **out)
        print(f"stage cap {cap}: initial {len(out['initial_patches'])} all {len(out['all_patches'])} "
              f"in {out['ref_seconds']:.1f}s")
    for cap in a.filter_stage:
        out = stage_golden(MVS2, imgs, seeds_to_tracks(seeds), cap, with_filter=True)
        np.savez_compressed(os.path.join(HERE, f"stage_filter_cap{cap}.npz"), **out)
        print(f"stage cap {cap} with filter_out_outlier: initial {len(out['initial_patches'])} "
              f"all {len(out['all_patches'])} removed lines {int(out['removed_lines'])} "
              f"in {out['ref_seconds']:.1f}s", flush=True)


if __name__ == "__main__":
    main()

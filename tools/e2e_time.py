"""End-to-end timing of the reference's pipeline on dinoRing (BASELINE configs
1/3/5): images -> SfM tracks (Harris/NCC front-end) -> MVS stage (100k pops)
-> PLY rows, on the GPU through the package, and the same pipeline through
the CPU oracle (sfm_oracle.c + mvs_oracle.c) on the host cores.  The two
must produce the same rows.  Prints one JSON line."""
import importlib, json, os, sys, time
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests/golden")
PKG = "simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd"
DATA = "/root/repo/data/dinoRing"
POPS = int(os.environ.get("E2E_POPS", "100000"))


class Args:
    img_dir = DATA
    img_type = "png"
    par_path = os.path.join(DATA, "dinoR_par.txt")
    scale = 10.0
    cell_size = 2
    desc_wid = 5
    debug = False
    nonSeq = False


def main():
    import contextlib, io
    out = {"pops": POPS}
    t0 = time.perf_counter()
    import torch
    assert torch.cuda.is_available()
    mvs = importlib.import_module(PKG)
    with contextlib.redirect_stdout(io.StringIO()):
        imgs = mvs.read_imgs(Args())
    t1 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        K, R, t = mvs.utils.pars_to_arrays(*mvs.read_pars(Args()), len(imgs))
    ctx = mvs.MvsContext(np.stack(imgs), K, R, t)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    gs = mvs.sfm.GlobalSet(0.01)
    with contextlib.redirect_stdout(io.StringIO()):
        mvs.sfm.StructureFromMotion(imgs, gs, Args(), 0.3, matcher=mvs.sfm.HarrisMatcher(ctx))
    off, ov, oxy = mvs.utils.tracks_to_arrays(gs.getInfo()[2])
    t3 = time.perf_counter()
    ini, allp, st = ctx.stage(off, ov, oxy, cell_size=2, scale=10.0, wid=5, max_pops=POPS)
    t4 = time.perf_counter()
    out.update({"gpu_read_imgs_s": t1 - t0, "gpu_context_s": t2 - t1, "gpu_sfm_s": t3 - t2,
                "gpu_mvs_stage_s": t4 - t3, "gpu_total_s": t4 - t0, "tracks": int(len(off) - 1),
                "initial": int(len(ini)), "all": int(len(allp)), "stage": st})
    # the same pipeline on the CPU oracle
    from oracle import oracle as orc
    sfm = mvs.sfm
    nth = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    c0 = time.perf_counter()
    rgb = np.stack(imgs)
    V, H, W = rgb.shape[:3]
    grays = [orc.gray_from_rgb(rgb[v]) for v in range(V)]
    locs = [sfm.desc_bounds_rc(orc.harris_points(g), H, W) for g in grays]

    def cpu_matcher(a, b):
        da, db = orc.descriptors(grays[a], locs[a]), orc.descriptors(grays[b], locs[b])
        b12 = orc.match_best(da, db, 0.5)[0]
        b21 = orc.match_best(db, da, 0.5)[0]
        m12 = np.array([j if j >= 0 and b21[j] == i else -1 for i, j in enumerate(b12)])
        src, dst = sfm.get_matches(locs[a], locs[b], m12)
        return src.astype(np.float32), dst.astype(np.float32), len(src)

    gs2 = sfm.GlobalSet(0.01)

    def cpu_pair(KA, RA, tA, KB, RB, tB, q, tr, e):
        return orc.sfm_pair(KA, RA, tA, KB, RB, tB, q, tr, e)

    real_pair = mvs._lib.sfm_pair
    mvs._lib.sfm_pair = cpu_pair          # the oracle's pair geometry for the CPU leg
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            sfm.StructureFromMotion(imgs, gs2, Args(), 0.3, matcher=cpu_matcher)
    finally:
        mvs._lib.sfm_pair = real_pair
    off2, ov2, oxy2 = mvs.utils.tracks_to_arrays(gs2.getInfo()[2])
    c1 = time.perf_counter()
    oini, oall, _ = orc.Scene(rgb, K, R, t).mvs_stage(off2, ov2, oxy2, scale=10.0, max_pops=POPS)
    c2 = time.perf_counter()
    out.update({"cpu_threads_sfm": nth, "cpu_sfm_s": c1 - c0, "cpu_mvs_stage_s_1thread": c2 - c1,
                "cpu_total_s": c2 - c0,
                "tracks_equal": bool(np.array_equal(off, off2) and np.array_equal(ov, ov2) and
                                     np.array_equal(oxy, oxy2)),
                "rows_equal": bool(np.array_equal(ini, oini) and np.array_equal(allp, oall))})
    print(json.dumps(out))


if __name__ == "__main__":
    main()

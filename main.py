"""Entry point with the reference's flags (main.py:33-42 of the reference):

    python main.py -img_p data/dinoRing -par_p data/dinoRing/dinoR_par.txt -t png -scale 10 \
                   -seeds tests/golden/seeds_dino.npz

The MVS stage (DensePointsWithMVS2, MVS2.py:176) runs on the GPU through
libmvs_amd.so and writes initial_patches.ply / all_patches.ply in the working
directory, like the reference.  Under torchrun (one process per GPU) the
expansion sweeps are sharded over the GPUs:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py -img_p ... -seeds ...

Tracks: without -seeds, StructureFromMotion (SFM.py:47-88) runs first with the
reference's Harris/NCC features (HarrisFeatures.py) matched on the GPU in
place of OpenCV's ORB + FLANN + RANSAC (absent from this image); with -seeds
FILE.npz (track_off, obs_view, obs_xy, the format tests/golden/make_seeds.py
and -save_tracks write) the tracks are read instead.
"""
import importlib
import os
import sys
from argparse import ArgumentParser

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_NAME = "simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd"
sys.path.insert(0, REPO)


def main(args, threshold=0.01, MIN_REPROJECTION_ERROR=0.3):
    mvs = importlib.import_module(PKG_NAME)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        # one process per GPU (torchrun): the expansion sweeps are sharded over
        # the ranks and exchanged with RCCL (parallel.stage_sharded)
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    imgs = mvs.read_imgs(args)
    if getattr(args, "seeds", None):
        global_set = mvs.SeedSet.load(args.seeds)
    else:
        # SfM.StructureFromMotion (main.py:28) with the Harris/NCC front-end on
        # the GPU in place of OpenCV's ORB/FLANN/RANSAC (sfm.py)
        global_set = mvs.sfm.GlobalSet(threshold=threshold)
        st = mvs.sfm.StructureFromMotion(imgs, global_set, args, MIN_REPROJECTION_ERROR)
        n_obs, n_pts, _ = global_set.getInfo()
        print(f"SfM: {st['pairs']} pairs, {st['correspondences']} correspondences, "
              f"{st['kept']} triangulated, {n_pts} tracks / {n_obs} observations")
    if getattr(args, "save_tracks", None) and (world == 1 or int(os.environ.get("RANK", "0")) == 0):
        import numpy as np
        off, view, xy = mvs.utils.tracks_to_arrays(global_set.getInfo()[2])
        np.savez(args.save_tracks, track_off=off, obs_view=view, obs_xy=xy)
    mvs.DensePointsWithMVS2(imgs, global_set, args, max_pops=getattr(args, "max_pops", 100000))
    st = mvs.MVS2.last_stats
    if world == 1 or int(os.environ.get("RANK", "0")) == 0:
        print("pops {pops} tests {tests} accepted {accepts} gpu-scored {scored} sweeps {sweeps}".format(**st))


if __name__ == "__main__":
    parser = ArgumentParser()
    parser.add_argument("-img_p", help="image directory", dest="img_dir", default=None)
    parser.add_argument("-par_p", help="parameter path", dest="par_path", default=None)
    parser.add_argument("-t", help="image file type", dest="img_type", default="ppm")
    parser.add_argument("-scale", help="scale", dest="scale", default=1, type=float)
    parser.add_argument("--debug", help="debug mode on", dest="debug", action="store_true")
    parser.add_argument("--nonSequence", help="", dest="nonSeq", action="store_true")
    parser.add_argument("-cell_size", help="", dest="cell_size", default=2, type=int)
    parser.add_argument("-desc_wid", help="", dest="desc_wid", default=5, type=int)
    parser.add_argument("-seeds", help="SfM tracks (npz: track_off, obs_view, obs_xy)",
                        dest="seeds", default=None)
    parser.add_argument("-max_pops", help="expansion pop cap (<= 100000)", dest="max_pops",
                        default=100000, type=int)
    parser.add_argument("--filter_outliers", dest="filter_outliers", action="store_true",
                        help="run CellTable.filter_out_outlier before the reconstruction (the "
                             "reference has the call commented out, MVS2.py:281)")
    parser.add_argument("-save_tracks", help="write the SfM tracks (npz) before the MVS stage",
                        dest="save_tracks", default=None)
    args = parser.parse_args()
    try:
        main(args)
    except RuntimeError as e:
        print("RuntimeError", e)
        sys.exit(1)

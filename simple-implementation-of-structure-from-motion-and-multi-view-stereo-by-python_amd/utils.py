"""Input / output formats of the MVS stage (utils.py and main.py of the reference).

read_pars   -- Middlebury *_par.txt cameras (utils.py:56-81)
read_imgs   -- sorted image list, RGB uint8 (main.py:7-20)
export2ply  -- x,y,z,red,green,blue float64 rows to a binary little-endian PLY
               (utils.py:249-251, pyntcloud's default .ply writer; the byte
               layout is unpinned: pyntcloud is absent from the image)
tracks_to_arrays -- GlobalSet.getInfo() tracks (GlobalSet.py:36-50) -> the flat
               arrays of the C-ABI (track_off, obs_view, obs_xy float32)
"""
import glob
import os

import numpy as np


def read_pars(args):
    """Same contract as utils.read_pars: dicts view -> K (3x3), R (3x3), t (3x1)."""
    print("get parameters from" + args.par_path)
    par_K, par_r, par_t = {}, {}, {}
    with open(args.par_path, "r") as f:
        lines = f.readlines()
    for i, line in enumerate(lines):
        if i == 0:
            continue
        tp = [float(v) for v in line.split()[1:]]
        par_K[i - 1] = np.array(tp[0:9]).reshape(3, 3)
        par_r[i - 1] = np.array(tp[9:18]).reshape(3, 3)
        par_t[i - 1] = np.array(tp[18:21]).reshape(3, 1)
    return par_K, par_r, par_t


def pars_to_arrays(par_K, par_r, par_t, n):
    K = np.stack([par_K[i] for i in range(n)]).astype(np.float64)
    R = np.stack([par_r[i] for i in range(n)]).astype(np.float64)
    t = np.stack([np.asarray(par_t[i]).reshape(3) for i in range(n)]).astype(np.float64)
    return K, R, t


def read_imgs(args):
    """glob(img_dir/*.img_type), sorted, decoded to RGB uint8 (main.py:7-20)."""
    from PIL import Image
    print("read images from " + args.img_dir + "/*." + args.img_type)
    files = sorted(glob.glob(args.img_dir + "/*." + args.img_type))
    print(files)
    return [np.asarray(Image.open(f).convert("RGB")).copy() for f in files]


def export2ply(points, colors, path="output"):
    """Write path + '.ply' with double properties x y z red green blue."""
    pts = np.asarray(points, np.float64).reshape(-1, 3)
    col = np.asarray(colors).reshape(-1, 3).astype(np.float64)
    data = np.hstack((pts, col))
    header = ("ply\nformat binary_little_endian 1.0\n"
              f"element vertex {len(data)}\n"
              "property double x\nproperty double y\nproperty double z\n"
              "property double red\nproperty double green\nproperty double blue\n"
              "end_header\n")
    with open(path + ".ply", "wb") as f:
        f.write(header.encode("ascii"))
        f.write(np.ascontiguousarray(data, "<f8").tobytes())


def read_ply(path):
    """Inverse of export2ply (tests, tools)."""
    with open(path, "rb") as f:
        raw = f.read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    n = int([ln for ln in raw[:end].decode().splitlines() if ln.startswith("element vertex")][0].split()[-1])
    return np.frombuffer(raw[end:], "<f8", count=n * 6).reshape(n, 6).copy()


def tracks_to_arrays(tracks):
    """[track.point2d_list = [(view, x, y), ...]] -> (track_off i64, obs_view i32, obs_xy f32)."""
    off, view, xy = [0], [], []
    for tr in tracks:
        for ob in tr.point2d_list:
            view.append(int(ob[0]))
            xy.append((np.float32(ob[1]), np.float32(ob[2])))
        off.append(len(view))
    return (np.array(off, np.int64), np.array(view, np.int32),
            np.array(xy, np.float32).reshape(-1, 2))


class SeedTrack:
    def __init__(self, obs):
        self.point2d_list = obs


class SeedSet:
    """Minimal GlobalSet stand-in built from flat track arrays (an SfM output file)."""

    def __init__(self, track_off, obs_view, obs_xy):
        self.tracks = [SeedTrack([(int(obs_view[o]), np.float32(obs_xy[o][0]), np.float32(obs_xy[o][1]))
                                  for o in range(track_off[k], track_off[k + 1])])
                       for k in range(len(track_off) - 1)]

    @classmethod
    def load(cls, path):
        z = np.load(path)
        return cls(z["track_off"], z["obs_view"], z["obs_xy"])

    def getInfo(self):
        return sum(len(t.point2d_list) for t in self.tracks), len(self.tracks), self.tracks

"""The reference's own CPU speed on this path, from the stage fixtures'
recorded wall times (gen_golden.py --stage / --filter-stage ran the
reference's DensePointsWithMVS2 single-threaded in the build container and
stored ref_seconds) and the number of photo tests those runs performed,
counted by the oracle run to the same pop cap (pinned bit-exact to those
fixtures: same rows, same pops).  Photo tests = seeding tests (MVS2.py:255)
+ expansion tests (MVS2.py:362).  Writes reference_timing.json for bench.py's
cpu_baseline.reference_python (the reference never travels to the GPU box).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, HERE)
from make_seeds import load_dino  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    imgs, K, R, t = load_dino(os.path.join(HERE, "..", "..", "data", "dinoRing"))
    sc = orc.Scene(np.stack(imgs), K, R, t)
    s = dict(np.load(os.path.join(HERE, "seeds_dino.npz")))
    # every seed track is a 2-view track: one seeding candidate, one photo test
    # each (MVS2.py:238-257)
    lens = np.diff(s["track_off"])
    assert (lens == 2).all()
    seed_tests = int(len(lens))
    runs = []
    for name in ("stage_cap200", "stage_cap2000", "stage_filter_cap200", "stage_filter_cap1000"):
        g = dict(np.load(os.path.join(HERE, name + ".npz")))
        cap = int(g["cap"])
        ini, allp, st = sc.mvs_stage(s["track_off"], s["obs_view"], s["obs_xy"], scale=10.0, max_pops=cap)
        assert np.array_equal(allp, g["all_patches"]) and st["pops"] == int(g["pops"])
        runs.append({"fixture": name + ".npz", "pops": cap, "expansion_tests": int(st["tests"]),
                     "seed_tests": seed_tests, "photo_tests": int(st["tests"]) + seed_tests,
                     "ref_seconds": float(g["ref_seconds"]),
                     "photo_tests_per_s": (int(st["tests"]) + seed_tests) / float(g["ref_seconds"])})
    json.dump({"note": "reference DensePointsWithMVS2 (MVS2.py:176-295), CPython single thread, "
                       "8-core Xeon build container, OpenCV stand-ins (SURVEY.md 8c); seconds "
                       "recorded by tests/golden/gen_golden.py when the fixture was generated",
               "runs": runs}, open(os.path.join(HERE, "reference_timing.json"), "w"), indent=1)
    print(json.dumps(runs, indent=1))


if __name__ == "__main__":
    main()

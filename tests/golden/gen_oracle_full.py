"""Full-run fixture: the oracle (oracle/mvs_oracle.c, pinned to the reference
at caps 200 and 2000 by test_oracle_golden.py) run to the reference's own
100,000-pop cap on dinoRing + seeds_dino.npz.  The reference itself would need
~10 h for this, so the full-length fixture is the
oracle's; only counts and checksums are committed (the rows are ~29 MB).

  python gen_oracle_full.py [cap] [views]   # views 47: BASELINE config 3's view
  count on the dinoRing subset (views 0-46, seeds restricted to them)."""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, HERE)
from make_seeds import load_dino, subset_seeds  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, "<f8").tobytes()).hexdigest()


def main(cap=100000, views=48):
    imgs, K, R, t = load_dino(os.path.join(HERE, "..", "..", "data", "dinoRing"))
    sc = orc.Scene(np.stack(imgs)[:views].copy(), K[:views].copy(), R[:views].copy(), t[:views].copy())
    s = dict(np.load(os.path.join(HERE, "seeds_dino.npz")))
    args = subset_seeds(s, views) if views < 48 else (s["track_off"], s["obs_view"], s["obs_xy"])
    t0 = time.time()
    ini, allp, st = sc.mvs_stage(*args, cell_size=2, scale=10.0, wid=5, max_pops=cap)
    dt = time.time() - t0
    out = {"cap": cap, "views": views, "oracle_seconds": dt, "n_initial": len(ini), "n_all": len(allp),
           "stats": st, "sha256_initial": digest(ini), "sha256_all": digest(allp),
           "sum_all": [float(x) for x in allp.sum(0)], "first_rows": allp[:5].tolist(),
           "last_rows": allp[-5:].tolist()}
    name = f"stage_oracle_cap{cap}.json" if views == 48 else f"stage_oracle_v{views}_cap{cap}.json"
    json.dump(out, open(os.path.join(HERE, name), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("first_rows", "last_rows")}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100000,
         int(sys.argv[2]) if len(sys.argv) > 2 else 48)

"""Merge rocprofv3 --pmc pass directories into a pmc.json (profiles/rNN/): the
per-launch counters of the scorer kernel (k_score_tab / k_score_mma*) for one bench
configuration.  bench.py reads this file to compute its roofline fractions.
usage: pmc_json.py OUT.json SCENE V WID N PMC_DIR"""
import collections
import csv
import glob
import json
import os
import sys

out, scene, V, wid, n, root = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"]][row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
hits = [k for k in acc if "k_score_mma" in k or "k_score_tab" in k]
if len(hits) != 1:
    sys.exit(f"scorer kernel ambiguous: {hits}")
k = hits[0]
per = {cn: sum(v.values()) / len(v) for cn, v in acc[k].items()}
db = json.load(open(out)) if os.path.exists(out) else {"entries": []}
db["entries"] = [e for e in db["entries"] if (e["scene"], e["V"], e["wid"], e["n"]) != (scene, V, wid, n)]
db["entries"].append({"scene": scene, "V": V, "wid": wid, "n": n, "kernel": k, "per_launch": per,
                      "source": os.path.normpath(root),
                      "notes": "rocprofv3 --pmc, one counter group per run (tools/pmc.sh); per-dispatch "
                               "averages; FETCH_SIZE/WRITE_SIZE in KiB (bench.py doubles FETCH_SIZE, "
                               "the gfx950 correction for 16-B-per-lane reads); SQ_ACTIVE_INST_VALU in "
                               "quad-cycles summed over all SIMDs"})
db["entries"].sort(key=lambda e: (e["scene"], e["wid"]))
json.dump(db, open(out, "w"), indent=1)
print(k[:80], {c: per[c] for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_ACTIVE_INST_VALU") if c in per})

"""Summarise rocprofv3 --pmc passes: per-kernel average of each counter per dispatch."""
import csv, glob, os, sys, collections, json
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        acc[k][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
out = {}
for k, cs in acc.items():
    # per dispatch sums (a counter can appear once per dimension instance)
    d = {}
    for cn, vals in cs.items():
        per = collections.defaultdict(float)
        for did, v in vals:
            per[did] += v
        d[cn] = sum(per.values()) / len(per)
    out[k] = d
for k, d in out.items():
    if "score" not in k and "bin" not in k:
        continue
    print(k[:70])
    for cn, v in sorted(d.items()):
        print(f"   {cn:24s} {v:16.1f}")
json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)

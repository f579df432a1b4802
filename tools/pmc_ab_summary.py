"""Mean per-dispatch PMC counters of the scorer kernels under a rocprofv3 output dir."""
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(dict)
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "k_score" not in k:
            continue
        per[(row["Dispatch_Id"], k)][row["Counter_Name"]] = per[(row["Dispatch_Id"], k)].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    for (d, k), cs in per.items():
        for c, v in cs.items():
            acc[k][c].append(v)
for k, cs in acc.items():
    print(k[:90])
    for c, vs in sorted(cs.items()):
        print(f"   {c:24s} {sum(vs) / len(vs):16.0f}  (n={len(vs)})")

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

# Per-launch HBM traffic of the dominant kernel for bench.py's roofline.traffic:
# rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
# half the bytes of 16-B-per-lane reads (MI355X_MICROARCH.md, HBM/rocprofv3
# section), so it is doubled; WRITE_SIZE is taken as is.
# usage: pmc_summary.py DIR [KERNEL_SUBSTR N WID V OUT.json]
if len(sys.argv) >= 7:
    ksub, n, wid, V, dst = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    hits = [k for k in out if ksub in k]
    if len(hits) != 1:
        sys.exit(f"kernel substring {ksub!r} matches {hits}")
    d = out[hits[0]]
    fetch = d["FETCH_SIZE"] * 1024 * 2
    write = d["WRITE_SIZE"] * 1024
    json.dump({"kernel": hits[0], "n": n, "wid": wid, "V": V,
               "fetch_bytes_corrected": fetch, "write_bytes": write,
               "bytes_per_launch": fetch + write,
               "bytes_per_candidate": (fetch + write) / n,
               "source": os.path.normpath(root),
               "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 16-B/lane reads), WRITE_SIZE KiB x1024"},
              open(dst, "w"), indent=1)
    print("traffic", hits[0][:60], (fetch + write) / 1e6, "MB per launch")

"""Summarise a gpu_r3.sh run: rocprof kernel averages and the bench line's key
figures.  usage: python tools/summ.py TAG"""
import csv
import json
import sys

tag = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/{tag}_kernel_stats.csv")):
    print(f"{r['Name'][:70]:72s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.2f} us")
try:
    d = json.loads(open(f"gpurun_out/{tag}_bench_full.log").read().strip().splitlines()[-1])
except (OSError, ValueError, IndexError):
    sys.exit(0)
r = d["roofline"]
print("value %.3f G  step %.1f us  kernel %.1f us  bound %s %.3f  hbm %.3f" % (
    d["value"] / 1e9, d["ms_per_step"] * 1e3, r["kernel_ms"] * 1e3, r["bound"], r["frac"],
    r["roofs"].get("hbm", {}).get("frac", float("nan"))))
for k in ("cold_sweep", "secondary", "stage", "ring256", "exchange"):
    v = d.get(k)
    if v:
        print(k, {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()
                  if not isinstance(vv, (dict, list)) and kk not in ("workload", "note", "unit")})

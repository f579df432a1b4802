"""Per-step timeline of the headline score call from a rocprofv3 kernel trace:
kernel durations and the idle gaps between consecutive kernels on the GPU.
usage: trace_gaps.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0] for r in rows]
# one step = k_bin ... k_score_fix; take the steps after warmup
steps, cur = [], []
for r, n in zip(rows, names):
    if n.startswith("k_bin") and cur:
        steps.append(cur)
        cur = []
    cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
steps.append(cur)
steps = [[x for x in s if x[0].startswith("k_")] for s in steps]
steps = [s for s in steps if any(n.startswith("k_score_mma") for n, _, _ in s) and len(s) <= 6]
dur = defaultdict(list)
gap = defaultdict(list)
span = []
for s in steps[5:]:
    span.append((s[-1][2] - s[0][1]) / 1e3)
    nxt = [x for x in steps if x[0][1] > s[-1][2]]
    if nxt:
        gap["(next step)"].append((nxt[0][0][1] - s[-1][2]) / 1e3)
    for i, (n, a, b) in enumerate(s):
        dur[n].append((b - a) / 1e3)
        if i:
            gap[n].append((a - s[i - 1][2]) / 1e3)
print(f"{len(steps) - 5} steps, first kernel start to last kernel end: {sum(span) / len(span):.1f} us")
if gap.get("(next step)"):
    g = sorted(gap["(next step)"])
    print(f"  idle from a step's last kernel to the next step's first: median {g[len(g) // 2]:.1f} us")
for n in dur:
    g = sum(gap[n]) / len(gap[n]) if gap[n] else 0.0
    print(f"  {n[:40]:40s} {sum(dur[n]) / len(dur[n]):8.1f} us   gap before {g:6.1f} us")

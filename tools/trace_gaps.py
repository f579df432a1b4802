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
steps = [s for s in steps if any(n.startswith("k_score_mma") for n, _, _ in s)]
dur = defaultdict(list)
gap = defaultdict(list)
span = []
for s in steps[5:]:
    span.append((s[-1][2] - s[0][1]) / 1e3)
    for i, (n, a, b) in enumerate(s):
        dur[n].append((b - a) / 1e3)
        if i:
            gap[n].append((a - s[i - 1][2]) / 1e3)
print(f"{len(steps) - 5} steps, first kernel start to last kernel end: {sum(span) / len(span):.1f} us")
for n in dur:
    g = sum(gap[n]) / len(gap[n]) if gap[n] else 0.0
    print(f"  {n[:40]:40s} {sum(dur[n]) / len(dur[n]):8.1f} us   gap before {g:6.1f} us")

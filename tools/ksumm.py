"""Kernel averages of a rocprofv3 kernel_stats.csv.  usage: python tools/ksumm.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else None]:
    print(f"{r['Name'][:70]:72s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.2f} us")

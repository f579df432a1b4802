"""Kernel averages of a rocprofv3 kernel_stats.csv.  usage: python tools/ksumm.py FILE"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:72s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.2f} us")

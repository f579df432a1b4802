#!/bin/bash
# Instruction-cache counters of the headline kernels (one rocprofv3 --pmc
# pass, time-limited); per-dispatch averages printed.  Usage (GPU box):
# bash tools/pmc_icache.sh TAG
export TMPDIR=/tmp
TAG=${1:-ic}
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 --no-stage --no-ring --no-overlap --comm-cus 0"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVES \
  -d gpurun_out/pmci_$TAG -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmci_$TAG.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/pmci_$TAG.log; exit $rc; }
python - gpurun_out/pmci_$TAG <<'PY'
import collections, csv, glob, os, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", row["Kernel_Name"])
        if m: acc[m.group(1)][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(k, "  ".join(f"{c} {sum(v) / len(v):.0f}" for c, v in sorted(d.items())))
PY
rm -rf gpurun_out/pmci_$TAG

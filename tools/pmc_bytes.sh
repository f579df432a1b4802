#!/bin/bash
# HBM-side bytes (FETCH_SIZE, WRITE_SIZE; TCC hits/misses) of every kernel of
# the headline step and the exchange's pack, one counter group per rocprofv3
# run.  Usage (GPU box): bash tools/pmc_bytes.sh TAG
export TMPDIR=/tmp
TAG=${1:-bytes}
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 --no-stage --no-ring --no-overlap --comm-cus 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmcb_$TAG/p$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmcb_${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/pmcb_${TAG}_p$i.log; exit $rc; }
done
python - gpurun_out/pmcb_$TAG <<'PY'
import collections, csv, glob, os, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(os.path.join(sys.argv[1], "p*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", row["Kernel_Name"])
        if m and m.group(1) in ("k_bin", "k_score_tab", "k_score_fix", "k_acc_pack", "k_moments", "k_build_scene"):
            acc[m.group(1)][row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:40s} {sum(v.values()) / len(v):16.1f} per dispatch ({len(v)} dispatches)")
PY
rm -rf gpurun_out/pmcb_$TAG

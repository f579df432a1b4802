#!/bin/bash
# Memory-pipe counters of the headline scorer, k_bin and k_acc_pack (TA/TD/TCP/SQ VMEM, HBM bytes), one counter
# group per rocprofv3 run, each time-limited; per-launch averages of the
# scorer printed.  Usage (GPU box): bash tools/pmc_mem.sh TAG [bench args]
export TMPDIR=/tmp
TAG=${1:-mem}; shift
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 --no-stage --no-ring --no-overlap --comm-cus 0 $@"
i=0
for grp in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmcm_$TAG/p$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmcm_${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/pmcm_${TAG}_p$i.log; exit $rc; }
done
python - gpurun_out/pmcm_$TAG <<'PY'
import collections, csv, glob, os, re, sys
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(os.path.join(sys.argv[1], "p*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        if "k_score_tab" in row["Kernel_Name"] or "k_bin" in row["Kernel_Name"] or "k_acc_pack" in row["Kernel_Name"]:
            k = re.search(r"(k_\w+)", row["Kernel_Name"]).group(1)
            acc[k][row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:40s} {sum(v.values()) / len(v):16.1f} per dispatch ({len(v)} dispatches)")
PY
rm -rf gpurun_out/pmcm_$TAG

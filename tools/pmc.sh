#!/bin/bash
# PMC passes for the bench's kernels: one counter group per rocprofv3 run
# (no trace domains besides the default kernel dispatches), each time-limited.
# Usage (GPU box): bash tools/pmc.sh TAG [bench args...]
export TMPDIR=/tmp
TAG=${1:-dev}; shift
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 --no-stage --no-ring --no-overlap --comm-cus 0 $@"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${PMC_EXTRA}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc_${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${TAG}_p$i.log; exit $rc; }
done
exit 0

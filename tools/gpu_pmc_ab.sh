#!/bin/bash
# LDS-side PMC counters of two scorer variants in one process (tools/ab_variants.py), one --pmc pass.
# usage: bash tools/gpu_pmc_ab.sh TAG "10 0" [wid]
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; VARS=$2; WID=${3:-5}
AB_WID=$WID timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES \
  -d gpurun_out/pmcab_$TAG -o run --output-format csv -- python tools/ab_variants.py $VARS > gpurun_out/pmcab_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmcab_$TAG.log; exit $rc; }
python tools/pmc_ab_summary.py gpurun_out/pmcab_$TAG > gpurun_out/pmcab_${TAG}_summary.txt; cat gpurun_out/pmcab_${TAG}_summary.txt

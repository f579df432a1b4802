#!/bin/bash
# Phase stamps of the scorers (diagnostic build, build_lib.py --stamps):
# k_score_mma on dinoRing at wid 5 and 3, k_score_mma_v on ring256 at wid 5.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TAG=${1:-diag}
LOG=gpurun_out/stamps_${TAG}.log
: > $LOG
for args in ${STAMP_RUNS:-"5:dino" "3:dino" "5:ring256"}; do
  timeout -k 10 180 python tools/stamps.py ${args%%:*} ${args##*:} >> $LOG 2>&1 || { tail -5 $LOG; exit 1; }
done
cat $LOG

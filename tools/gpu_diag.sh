#!/bin/bash
# Diagnostics of the scorer: phase stamps (diagnostic build) and PMC passes.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-diag}
timeout -k 10 120 python tools/stamps.py 5 > gpurun_out/stamps_${TAG}.log 2>&1 || { tail -5 gpurun_out/stamps_${TAG}.log; exit 1; }
timeout -k 10 120 python tools/stamps.py 3 >> gpurun_out/stamps_${TAG}.log 2>&1 || { tail -5 gpurun_out/stamps_${TAG}.log; exit 1; }
cat gpurun_out/stamps_${TAG}.log
if [ -n "$PMC" ]; then
  bash tools/pmc.sh $TAG || exit 1
  python tools/pmc_summary.py gpurun_out/pmc_$TAG k_score_mma 1048576 5 48 gpurun_out/pmc_traffic_$TAG.json > gpurun_out/pmc_${TAG}_summary.txt 2>&1
  grep -A30 "k_score_mma" gpurun_out/pmc_${TAG}_summary.txt | head -30
fi

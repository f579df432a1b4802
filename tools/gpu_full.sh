#!/bin/bash
# Full GPU round-trip: parity tests, bench (+ CPU baseline), rocprof kernel stats, PMC traffic.
# Usage (on the GPU box): bash tools/gpu_full.sh TAG [bench args...]
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dev}; shift
bash tools/gpu_check.sh $TAG "$@" || exit 1
bash tools/pmc.sh $TAG "$@" || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG ${PMC_KERNEL:-k_score_tiled5} 1048576 5 48 gpurun_out/pmc_traffic_$TAG.json > gpurun_out/pmc_${TAG}_summary.txt 2>&1
tail -5 gpurun_out/pmc_${TAG}_summary.txt

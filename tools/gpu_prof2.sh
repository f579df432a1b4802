#!/bin/bash
# Round-2 profile of the matrix-core scorer: rocprof kernel stats (dino), the
# counter list, PMC passes (dino), ring256 bench + kernel stats.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -c1-160 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
bash tools/pmc.sh $TAG || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG k_score_mma 1048576 5 48 gpurun_out/pmc_traffic_$TAG.json > gpurun_out/pmc_${TAG}_summary.txt 2>&1
tail -3 gpurun_out/pmc_${TAG}_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ring -o run --output-format csv -- python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}_ring.log 2>&1
rc=$?; echo "ring prof rc=$rc"; tail -1 gpurun_out/prof_${TAG}_ring.log | cut -c1-300; cut -c1-160 gpurun_out/prof_${TAG}_ring/run_kernel_stats.csv | head -12
exit $rc

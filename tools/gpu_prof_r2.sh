#!/bin/bash
# Round-2 profiles: rocprof kernel stats of the full bench (headline, cold
# sweep, wid 3, stage, ring256), then PMC passes for the scorer at dino wid 5,
# dino wid 3 and ring256 wid 5 -> gpurun_out/pmc.json (copy to profiles/r02/).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r2}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -c1-160 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -14; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_$TAG.log; exit $rc; }
rm -f gpurun_out/pmc.json
bash tools/pmc.sh ${TAG}_w5 || exit 1
python tools/pmc_json.py gpurun_out/pmc.json dino 48 5 1048576 gpurun_out/pmc_${TAG}_w5 || exit 1
bash tools/pmc.sh ${TAG}_w3 --wid 3 || exit 1
python tools/pmc_json.py gpurun_out/pmc.json dino 48 3 1048576 gpurun_out/pmc_${TAG}_w3 || exit 1
if [ -z "$NO_RING_PMC" ]; then
  bash tools/pmc.sh ${TAG}_ring --scene ring256 || exit 1
  python tools/pmc_json.py gpurun_out/pmc.json ring256 256 5 1048576 gpurun_out/pmc_${TAG}_ring || exit 1
fi
exit 0

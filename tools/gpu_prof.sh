#!/bin/bash
# Profiles of a round (TAG, default r6): rocprof kernel stats of the full bench (headline, cold
# sweep, wid 3, stage, ring256), then PMC passes for the scorer at dino wid 5,
# dino wid 3 and ring256 wid 5 -> gpurun_out/pmc.json (copy to profiles/rNN/).
# Raw pass directories are reduced to the scorer's rows (gpurun_out/ must stay
# under the copy-back limit).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r6}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -c1-160 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -14; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_$TAG.log; exit $rc; }
cp gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/kernel_stats_$TAG.csv && rm -rf gpurun_out/prof_$TAG
# the headline alone (every scorer launch is a 2^20 sweep, so its rocprof
# average is comparable with the bench's HIP-event kernel_ms)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profh_$TAG -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-stage --no-ring --secondary-wid 0 > gpurun_out/profh_$TAG.log 2>&1
rc=$?; echo "headline prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/profh_$TAG.log; exit $rc; }
cp gpurun_out/profh_$TAG/run_kernel_stats.csv gpurun_out/kernel_stats_headline_$TAG.csv && rm -rf gpurun_out/profh_$TAG
[ -n "$HEADLINE_ONLY" ] && exit 0
rm -f gpurun_out/pmc.json
reduce() {   # keep the scorer's counter rows of a pass set, drop the rest
  head -1 $(ls $1/p1/run_counter_collection.csv) > $1_scorer.csv
  for f in $1/p*/run_counter_collection.csv; do grep -E "k_score_mma|k_score_tab|k_bin" "$f" >> $1_scorer.csv || true; done
  rm -rf $1
}
bash tools/pmc.sh ${TAG}_w5 || exit 1
python tools/pmc_json.py gpurun_out/pmc.json dino 48 5 1048576 gpurun_out/pmc_${TAG}_w5 || exit 1
reduce gpurun_out/pmc_${TAG}_w5
bash tools/pmc.sh ${TAG}_w3 --wid 3 || exit 1
python tools/pmc_json.py gpurun_out/pmc.json dino 48 3 1048576 gpurun_out/pmc_${TAG}_w3 || exit 1
reduce gpurun_out/pmc_${TAG}_w3
if [ -z "$NO_RING_PMC" ]; then
  bash tools/pmc.sh ${TAG}_ring --scene ring256 || exit 1
  python tools/pmc_json.py gpurun_out/pmc.json ring256 256 5 1048576 gpurun_out/pmc_${TAG}_ring || exit 1
  reduce gpurun_out/pmc_${TAG}_ring
fi
du -sh gpurun_out
exit 0

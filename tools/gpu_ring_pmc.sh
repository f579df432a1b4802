#!/bin/bash
# PMC passes + traffic summary for the ring256 (V = 256) tiled view-group scorer.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc.sh ring --scene ring256 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_ring k_score_tiledg 1048576 5 256 gpurun_out/pmc_traffic_ring.json > gpurun_out/pmc_ring_summary.txt 2>&1
rc=$?; tail -4 gpurun_out/pmc_ring_summary.txt; exit $rc

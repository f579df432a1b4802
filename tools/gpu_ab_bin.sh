#!/bin/bash
# A/B of the binning path: k_bin_fused (default) vs k_bin + k_tile_scan + k_scatter
# (MVS_BIN_FUSED=0): GPU tests, headline-only bench lines, rocprof stats of both.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -60; exit $rc; }
B="--no-stage --no-ring --secondary-wid 0 --steps 50"
timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_fused.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_fused.log | cut -c1-260
MVS_BIN_FUSED=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_3k.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_3k.log | cut -c1-260
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python bench.py $B > gpurun_out/${T}_prof.log 2>&1 || exit $?
find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/${T}_kernel_stats.csv | cut -c1-140 | head -8

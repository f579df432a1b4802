#!/bin/bash
# GPU tests, the headline-only bench line and its rocprof kernel stats (csv),
# the full default bench line last (TAG names the outputs).
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -60; exit $rc; }
B="--no-stage --no-ring --secondary-wid 0 --steps 50 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py $B > gpurun_out/${T}_prof.log 2>&1 || exit $?
find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
rm -rf gpurun_out/${T}_prof
cut -d, -f1-4 gpurun_out/${T}_kernel_stats.csv | cut -c1-140 | head -8
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_full.log 2>&1 || exit $?
  tail -1 gpurun_out/${T}_bench_full.log | cut -c1-400
fi

#!/bin/bash
# Round-3 GPU check: the GPU tests (-s: timing prints), then the headline-only
# bench line under rocprofv3 kernel stats; TAG names the outputs.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r3}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; }
fi
B="--no-stage --no-ring --secondary-wid 0 --steps 50 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py $B > gpurun_out/${T}_prof.log 2>&1 || exit $?
find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
rm -rf gpurun_out/${T}_prof
cut -d, -f1-4 gpurun_out/${T}_kernel_stats.csv | cut -c1-140 | head -8
tail -1 gpurun_out/${T}_prof.log | cut -c1-300
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_full.log 2>&1 || exit $?
  tail -1 gpurun_out/${T}_bench_full.log | cut -c1-400
fi

#!/bin/bash
# Round-5 closing run: GPU tests, smoke(), the counter list of the box,
# gpu_prof_r5.sh (rocprof stats, PMC passes -> profiles/r05/pmc.json), the
# default bench line.  TAG names the outputs.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out profiles/r05
T=${TAG:-r5z}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -2 gpurun_out/${T}_smoke.log
fi
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1; echo "counter list rc=$?"
bash tools/gpu_prof_r5.sh $T || exit $?
cp gpurun_out/pmc.json profiles/r05/pmc.json && cp gpurun_out/pmc.json gpurun_out/${T}_pmc.json
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_full.log 2>&1 || { tail -5 gpurun_out/${T}_bench_full.log; exit 1; }
tail -1 gpurun_out/${T}_bench_full.log | cut -c1-400

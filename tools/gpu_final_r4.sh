#!/bin/bash
# Round-4 closing run: GPU tests, smoke(), PMC passes of the scorer (dino wid
# 5 / wid 3, ring256) -> profiles/r04/pmc.json (the bench's roofline source),
# rocprof kernel stats of the full bench and of the headline alone, then the
# default bench line.  TAG names the outputs.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out profiles/r04
T=${TAG:-r4z}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -2 gpurun_out/${T}_smoke.log
fi
bash tools/gpu_prof_r4.sh $T || exit $?
cp gpurun_out/pmc.json profiles/r04/pmc.json && cp gpurun_out/pmc.json gpurun_out/${T}_pmc.json
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_full.log 2>&1 || { tail -5 gpurun_out/${T}_bench_full.log; exit 1; }
tail -1 gpurun_out/${T}_bench_full.log | cut -c1-400

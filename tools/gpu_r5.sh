#!/bin/bash
# Round-5 GPU call: tests (PYTEST_K selects), the overlap probe (+ a kernel
# trace of it), and the default bench line.  TAG names the outputs; NO_TESTS,
# NO_PROBE, NO_BENCH skip parts.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r5}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -2 gpurun_out/${T}_smoke.log
fi
if [ -z "$NO_PROBE" ]; then
  timeout -k 10 300 python -u tools/overlap_probe.py ${PROBE_ARGS} > gpurun_out/${T}_probe.log 2>&1 || { tail -20 gpurun_out/${T}_probe.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_probe.log
  if [ -n "$TRACE" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_$T -o run --output-format csv -- python tools/overlap_probe.py ${TRACE} --steps 8 > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
    f=$(find gpurun_out/trace_$T -name '*kernel_trace.csv' | head -1)
    cp "$f" gpurun_out/${T}_kernel_trace.csv && rm -rf gpurun_out/trace_$T
    python tools/overlap_timeline.py gpurun_out/${T}_kernel_trace.csv ${TL_ARGS:-0 400} > gpurun_out/${T}_timeline.txt
    head -60 gpurun_out/${T}_timeline.txt
  fi
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 1; }
  tail -1 gpurun_out/${T}_bench.log | cut -c1-600
fi

#!/bin/bash
# What the driver runs at round end: GPU tests, smoke(), the default bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/re_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/re_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/re_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/re_bench.log 2>&1; rc=$?; tail -1 gpurun_out/re_bench.log | cut -c1-300; exit $rc

#!/bin/bash
# GPU box run: full -m gpu suite, then the default bench line (each step time-limited)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/t_gpu.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/t_gpu.log | head -80; exit $rc; }
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/b.log 2>&1
rc=$?; tail -3 gpurun_out/b.log; exit $rc

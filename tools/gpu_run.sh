#!/bin/bash
# GPU box run: full -m gpu suite, then the bench line (each step time-limited)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/t_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b.log 2>&1
rc=$?; tail -3 gpurun_out/b.log; exit $rc

#!/bin/bash
# round 2: first run of the matrix-core scorer -- new-path tests, then a short bench
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_paths.py -x -v --timeout 180 --timeout-method thread > gpurun_out/t_paths.log 2>&1
rc=$?; tail -25 gpurun_out/t_paths.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b.log 2>&1
rc=$?; tail -3 gpurun_out/b.log; exit $rc

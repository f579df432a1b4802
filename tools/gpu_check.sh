#!/bin/bash
# GPU round-trip used during development: parity tests, then bench + rocprof stats.
# Usage (on the GPU box): bash tools/gpu_check.sh TAG [bench args...]
export TMPDIR=/tmp
TAG=${1:-dev}; shift
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 5000 "$@" > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -c1-150 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -7

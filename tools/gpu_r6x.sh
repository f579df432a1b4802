#!/bin/bash
# Round 6, last session: k_moments with all loads in flight and bank-friendly
# LDS pitches -- the GPU tests, a rocprof kernel-stats pass of the default
# bench (k_moments per scene, k_build_scene, the step kernels) and its line.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r6x_pytest.log
[ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/r6x_pytest.log | head -60; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6x -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/r6x_bench_prof.log 2>&1 || { tail -5 gpurun_out/r6x_bench_prof.log; exit 1; }
f=$(find gpurun_out/prof_r6x -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r6x_kernel_stats_full.csv; rm -rf gpurun_out/prof_r6x
python tools/ksumm.py gpurun_out/r6x_kernel_stats_full.csv 12
python tools/ab_line.py gpurun_out/r6x_bench_prof.log "r6x"
grep -o '"cold_sweep": {[^}]*}' gpurun_out/r6x_bench_prof.log

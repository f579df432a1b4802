#!/bin/bash
# Whole MVS stage (seeding + 100k-pop expansion + output order) timing and kernel stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/stage_time.py 2000 100000 > gpurun_out/stage_time.log 2>&1; rc=$?; cat gpurun_out/stage_time.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stage -o run --output-format csv -- python tools/stage_time.py 100000 > gpurun_out/prof_stage.log 2>&1; rc=$?
echo "prof rc=$rc"; cut -c1-160 gpurun_out/prof_stage/run_kernel_stats.csv | head -12; exit $rc

#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "view_groups or view_count" --timeout 300 > gpurun_out/pytest_new.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_new.log; [ $rc -ne 0 ] && exit $rc
MVS_STAGE_TIMES=1 timeout -k 10 300 python tools/stage_time.py 100000 100000 > gpurun_out/stage_times.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/stage_times.log; exit $rc

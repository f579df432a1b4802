#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sfm.py -x -v -m gpu --timeout 300 > gpurun_out/pytest_sfm.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_sfm.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/sfm_time.py > gpurun_out/sfm_time.log 2>&1; rc=$?; tail -2 gpurun_out/sfm_time.log; exit $rc

#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "mask_words or view_count or view_groups" --timeout 300 > gpurun_out/pt_stress.log 2>&1; rc=$?; tail -2 gpurun_out/pt_stress.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/stress_score.py > gpurun_out/stress.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/stress.log | tail -8; exit $rc

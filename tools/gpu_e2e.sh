#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/e2e_time.py > gpurun_out/e2e.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/e2e.log | tail -3; exit $rc

#!/bin/bash
# A/B of k_score_tiled4 (variant 11) against k_score_tiled3 (variant 0), wid 5 and 3, then the GPU tests.
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_WID=5 timeout -k 10 300 python tools/ab_variants.py 0 11 > gpurun_out/ab_t4_w5.log 2>&1 || exit 1
AB_WID=3 timeout -k 10 300 python tools/ab_variants.py 0 11 > gpurun_out/ab_t4_w3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_t4_w5.log gpurun_out/ab_t4_w3.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/t4_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/t4_pytest.log; exit $rc

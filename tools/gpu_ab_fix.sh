#!/bin/bash
# A/B: guard lanes decided inside k_score_tiled3 (variant 0) vs 256-block k_score_fix grid (variant 13) vs 16 blocks (variant 0); GPU tests.
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_WID=5 timeout -k 10 300 python tools/ab_variants.py 13 0 > gpurun_out/ab_fix_w5.log 2>&1 || exit 1
AB_WID=3 timeout -k 10 300 python tools/ab_variants.py 13 0 > gpurun_out/ab_fix_w3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_fix_w5.log gpurun_out/ab_fix_w3.log
timeout -k 10 200 python tools/fix_count.py > gpurun_out/fix_count2.log 2>&1; grep -v amdgpu.ids gpurun_out/fix_count2.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/fix_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/fix_pytest.log; exit $rc

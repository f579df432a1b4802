#!/bin/bash
# A/B: k_score_tiled5 (row-streamed, 8-wave workgroups; variant 14 = 6 waves/SIMD, 15 = 8) vs k_score_tiled3 (0).
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_WID=3 timeout -k 10 300 python tools/ab_variants.py 10 14 15 > gpurun_out/ab_t5_w3.log 2>&1 || exit 1
AB_WID=5 timeout -k 10 300 python tools/ab_variants.py 10 14 15 > gpurun_out/ab_t5_w5.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_t5_w3.log gpurun_out/ab_t5_w5.log

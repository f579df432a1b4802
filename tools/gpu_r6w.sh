#!/bin/bash
# Round 6, last session: the exec-skip variant of the scorer's masked binary64
# sum (MVS_F64_SKIP) -- parity of the bench sweep under it, the headline-only
# A/B and rocprof stats -- then the step's HBM byte counters (pmc_bytes.sh).
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
L=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd_skip.so
MVS_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bench_sweep_full_size or bench_batch" > gpurun_out/r6w_skip_parity.log 2>&1 || { tail -30 gpurun_out/r6w_skip_parity.log; exit 1; }
tail -1 gpurun_out/r6w_skip_parity.log
NO_TESTS=1 VARIANTS=skip PROF=1 TAG=r6w bash tools/gpu_r6.sh || exit 1
bash tools/pmc_bytes.sh r6w > gpurun_out/r6w_pmc_bytes.log 2>&1; rc=$?; cat gpurun_out/r6w_pmc_bytes.log; exit $rc

#!/bin/bash
# k_score_mma_v phase stamps on ring256 (wid 5) for the stamps builds named in VARIANTS
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
D=simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
LOG=gpurun_out/ring_stamps_${TAG:-x}.log
: > $LOG
for v in ${VARIANTS:-new}; do
  echo "== $v" >> $LOG
  STAMPS_LIB=$PWD/$D/libmvs_amd_stamps_$v.so timeout -k 10 240 python tools/stamps.py 5 ring256 >> $LOG 2>&1 || { tail -5 $LOG; exit 1; }
done
grep -v amdgpu.ids $LOG

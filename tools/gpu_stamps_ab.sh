#!/bin/bash
# A/B of k_score_mma phase stamps: libmvs_amd_stamps_old.so vs _new.so (dino wid 5, 3)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
D=simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
LOG=gpurun_out/stamps_ab_${TAG:-x}.log
: > $LOG
for v in ${VARIANTS:-old new}; do
  for w in ${WIDS:-5 3}; do
    STAMPS_LIB=$PWD/$D/libmvs_amd_stamps_$v.so timeout -k 10 180 python tools/stamps.py $w dino >> $LOG 2>&1 || { tail -5 $LOG; exit 1; }
  done
done
grep -v amdgpu.ids $LOG

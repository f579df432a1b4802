#!/bin/bash
# A/B library variant: libmvs_amd_<name>.so built with extra flags
# (e.g. tools/build_variant.sh b8 -DMVS_BIN_PER=8); run with MVS_LIB=... or
# VARIANTS=<name> tools/gpu_ab.sh.  Variants are scratch: delete them after.
D=$(cd "$(dirname "$0")/.." && pwd)/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
N=$1; shift
cd $D/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -ffp-contract=off -fno-fast-math -Wno-unused-function "$@" \
  -o $D/libmvs_amd_$N.so mvs_kernels.hip mvs_score_tab.hip sfm_kernels.hip mvs_engine.cpp

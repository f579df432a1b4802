# usage: bash tools/gpu_ab.sh "0 4 5" [wid]
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_WID=${2:-5} timeout -k 10 300 python tools/ab_variants.py $1 > gpurun_out/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab.log | tail -12; exit $rc

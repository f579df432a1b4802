# parity tests under MVS_VARIANT=$1, then A/B of "$2" (wid 5 and 3)
export TMPDIR=/tmp
mkdir -p gpurun_out
MVS_VARIANT=$1 timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_v$1.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_v$1.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_v$1.log | head -10; exit $rc; }
AB_WID=5 timeout -k 10 300 python tools/ab_variants.py $2 > gpurun_out/ab_v5.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_v5.log | tail -8; [ $rc -ne 0 ] && exit $rc
AB_WID=3 timeout -k 10 300 python tools/ab_variants.py $2 > gpurun_out/ab_v3.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_v3.log | tail -8; exit $rc

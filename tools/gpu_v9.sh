export TMPDIR=/tmp
mkdir -p gpurun_out
MVS_VARIANT=9 timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_v9.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_v9.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_v9.log | head -10; exit $rc; }
AB_WID=5 timeout -k 10 300 python tools/ab_variants.py 0 9 > gpurun_out/ab_v5.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_v5.log | tail -4; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_stamps2.sh 9

export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/ubench/mfma_layout > gpurun_out/mfma_layout.log 2>&1; rc=$?; cat gpurun_out/mfma_layout.log; [ $rc -ne 0 ] && exit $rc
MVS_VARIANT=6 timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_mfma.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_mfma.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_variants.py 0 6 > gpurun_out/ab_mfma.log 2>&1; rc=$?; cat gpurun_out/ab_mfma.log | tail -6; [ $rc -ne 0 ] && exit $rc
AB_WID=3 timeout -k 10 300 python tools/ab_variants.py 0 6 > gpurun_out/ab_mfma3.log 2>&1; rc=$?; cat gpurun_out/ab_mfma3.log | tail -6; exit $rc

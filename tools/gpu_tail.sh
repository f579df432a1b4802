D=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
timeout -k 10 180 python tools/stamps_tab.py 5 > gpurun_out/stamps_tail2.log 2>&1 || { tail -5 gpurun_out/stamps_tail2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_tail2.log | tail -12
MVS_LIB=$D/libmvs_amd_ts512.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bench_sweep_full_size or score_records or in_kernel or table_cutoff or skewed or stage" > gpurun_out/ts512_pytest.log 2>&1 || { tail -30 gpurun_out/ts512_pytest.log; exit 1; }
tail -1 gpurun_out/ts512_pytest.log
TAG=r5v NO_TESTS=1 NO_UBENCH=1 LAYOUTS= VARIANTS="ts256 ts512" PROF_VARIANTS=1 bash tools/gpu_r5d.sh

D=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
MVS_LIB=$D/libmvs_amd_w10.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bench_sweep_full_size or score_records or table_cutoff or skewed or stage or view_groups" > gpurun_out/w10_pytest.log 2>&1 || { tail -30 gpurun_out/w10_pytest.log; exit 1; }
tail -1 gpurun_out/w10_pytest.log
TAG=r5wv NO_TESTS=1 NO_UBENCH=1 LAYOUTS= VARIANTS="w10 c768" PROF_VARIANTS=1 bash tools/gpu_r5d.sh

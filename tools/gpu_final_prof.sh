#!/bin/bash
# rocprof kernel stats: ring256 (view-group scorer v2) and the SfM front-end.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ring2 -o run --output-format csv -- python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ring2.log 2>&1
rc=$?; echo "ring prof rc=$rc"; cut -c1-150 gpurun_out/prof_ring2/run_kernel_stats.csv | head -6; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ring2f -o run --output-format csv -- python bench.py --scene ring256 --steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 > gpurun_out/pmc_ring2f.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_ring2w -o run --output-format csv -- python bench.py --scene ring256 --steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 > gpurun_out/pmc_ring2w.log 2>&1; rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sfm -o run --output-format csv -- python tools/sfm_time.py > gpurun_out/prof_sfm.log 2>&1
rc=$?; echo "sfm prof rc=$rc"; cut -c1-150 gpurun_out/prof_sfm/run_kernel_stats.csv | head -10; exit $rc

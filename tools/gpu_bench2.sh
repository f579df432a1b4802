export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_dino.log 2>&1; rc=$?; tail -1 gpurun_out/bench_dino.log | cut -c1-2500; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --scene ring256 --steps 20 --warmup 3 > gpurun_out/bench_ring.log 2>&1; rc=$?; tail -1 gpurun_out/bench_ring.log | cut -c1-2500; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ring -o run --output-format csv -- python bench.py --scene ring256 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ring.log 2>&1; rc=$?; cut -c1-150 gpurun_out/prof_ring/run_kernel_stats.csv | head -6; exit $rc

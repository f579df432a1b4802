# bench + rocprof kernel stats: bash tools/gpu_prof.sh TAG [bench args]
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dev}; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_$TAG.log | cut -c1-300; cut -c1-150 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -9; exit $rc

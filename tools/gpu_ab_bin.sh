#!/bin/bash
# A/B of k_bin's candidates per thread (MVS_BIN_PER 1/2/4/8): one rocprof
# kernel-stats run per setting (the choice is read once per process).
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 4 2 1 8; do
  MVS_BIN_PER=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abbin_$p -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --secondary-wid 0 > gpurun_out/abbin_$p.log 2>&1 || exit 1
  echo "MVS_BIN_PER=$p"; grep -h "k_bin\|k_scatter" gpurun_out/abbin_$p/run_kernel_stats.csv | cut -c1-120
  tail -1 gpurun_out/abbin_$p.log | cut -c1-300
done

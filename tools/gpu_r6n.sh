#!/bin/bash
# Round-6 A/B: band queues (k_score_tab, k_score_mma_v) and the binary64
# re-decision of guard-band pairs; parity subsets on each variant, ring256
# bench for the view-group scorer's variant.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
D=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
for v in bands d64g vbands; do
  MVS_LIB=$D/libmvs_amd_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -x -q --timeout 300 --timeout-method thread \
    -k "bench_sweep_full_size or threshold_on_reference or vs_oracle_bench_batch or ring256 or view_groups or dense_tile or skewed" > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
done
NO_TESTS=1 PROF=1 REPS=2 SWID=3 VARIANTS="bands d64g" bash tools/gpu_r6.sh || exit 1
for rep in 1 2; do for v in main vbands; do
  L=$D/libmvs_amd.so; [ $v != main ] && L=$D/libmvs_amd_$v.so
  MVS_LIB=$L timeout -k 10 300 python bench.py --scene ring256 --no-stage --no-ring --secondary-wid 0 --steps 50 --no-cpu-baseline --no-overlap > gpurun_out/${TAG}_ring_$v$rep.json 2>gpurun_out/${TAG}_ring.err || { tail -5 gpurun_out/${TAG}_ring.err; exit 1; }
  python tools/ab_line.py gpurun_out/${TAG}_ring_$v$rep.json "ring256 $v rep $rep" | tee -a gpurun_out/${TAG}_ab.log
done; done

#!/bin/bash
# Round-6 A/B (after the band queues became the default): the full GPU suite,
# the binary64 re-decision (d64g) and k_bin at 2 candidates per thread (bin2)
# against the library, parity subsets on the variants, the N = 1 step with
# the pack on the exchange's stream (--pack-on-comm).
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
D=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
T=${TAG:-r6o}
for v in d64g bin2; do
  MVS_LIB=$D/libmvs_amd_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -x -q --timeout 300 --timeout-method thread \
    -k "bench_sweep_full_size or threshold_on_reference or vs_oracle_bench_batch or dense_tile or skewed or edge" > gpurun_out/${T}_pytest_$v.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${T}_pytest_$v.log)"
done
TAG=$T PROF=1 REPS=2 SWID=3 VARIANTS="d64g bin2" bash tools/gpu_r6.sh || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-stage --no-ring --secondary-wid 0 --steps 100 --no-cpu-baseline --no-overlap --pack-on-comm > gpurun_out/${T}_b_poc$rep.json 2>gpurun_out/${T}_b.err || { tail -5 gpurun_out/${T}_b.err; exit 1; }
  python tools/ab_line.py gpurun_out/${T}_b_poc$rep.json "pack-on-comm rep $rep" | tee -a gpurun_out/${T}_ab.log
done

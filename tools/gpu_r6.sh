#!/bin/bash
# Round-6 iteration on one box: GPU tests (NO_TESTS=1 skips), the
# headline-only bench alternating the library and VARIANTS
# (libmvs_amd_<name>.so from build_variant.sh) REPS times each, a rocprof
# kernel-stats pass per library (PROF=1), then EXTRA (a command line).
# TAG names the outputs under gpurun_out/.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r6}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${T}_pytest.log
  if [ $rc -ne 0 ]; then grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; fi
fi
B="--no-stage --no-ring --secondary-wid ${SWID:-0} --steps 100 --no-cpu-baseline --no-overlap ${BENCH_ARGS}"
L0=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd.so
for rep in $(seq 1 ${REPS:-2}); do
  for v in main ${VARIANTS}; do
    L=$L0; [ $v != main ] && L=${L0%.so}_$v.so
    MVS_LIB=$L timeout -k 10 300 python bench.py $B > gpurun_out/${T}_b_$v$rep.json 2>gpurun_out/${T}_b.err || { tail -5 gpurun_out/${T}_b.err; exit 1; }
    python tools/ab_line.py gpurun_out/${T}_b_$v$rep.json "$v rep $rep" | tee -a gpurun_out/${T}_ab.log
  done
done
if [ -n "$PROF" ]; then
for v in main ${VARIANTS}; do
  L=$L0; [ $v != main ] && L=${L0%.so}_$v.so
  S=$T; [ $v != main ] && S=${T}_$v
  MVS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$S -o run --output-format csv -- python bench.py $B > gpurun_out/${S}_prof.log 2>&1 || { tail -5 gpurun_out/${S}_prof.log; exit 1; }
  f=$(find gpurun_out/prof_$S -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/${S}_kernel_stats.csv
  rm -rf gpurun_out/prof_$S
  echo "== $v (rocprof)" | tee -a gpurun_out/${T}_ab.log
  python tools/ksumm.py gpurun_out/${S}_kernel_stats.csv 8 | tee -a gpurun_out/${T}_ab.log
done
fi
if [ -n "$EXTRA" ]; then bash -c "$EXTRA" || exit 1; fi

#!/bin/bash
# Same-box A/B of the ring256 headline (k_score_mma_v, config 4): the library
# against $VARIANTS (a library variant name, or tab / mma for MVS_SCORE_KERNEL),
# twice each, plus the GPU tests named by PYTEST_K.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r4r}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -60; exit $rc; }
fi
B="--scene ring256 --no-stage --no-ring --secondary-wid 0 --steps 10 --warmup 2 --no-cpu-baseline --no-overlap"
: > gpurun_out/${T}_ab.log
for rep in 1 2; do
  for v in main ${VARIANTS}; do
    L=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd.so
    KM=
    case $v in main) ;; tab|mma) KM=$v ;; *) L=${L%.so}_$v.so ;; esac
    MVS_SCORE_KERNEL=$KM MVS_LIB=$L timeout -k 10 300 python bench.py $B > gpurun_out/${T}_b_$v.json 2>gpurun_out/${T}_b.err || { tail -5 gpurun_out/${T}_b.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/${T}_b_$v.json').read().strip().splitlines()[-1])
print('$v rep $rep: %.1f M cand/s  step %.1f us  kernel %.1f us (%s)' % (d['value']/1e6, d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['kernel']))" | tee -a gpurun_out/${T}_ab.log
  done
done

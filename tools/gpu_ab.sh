#!/bin/bash
# Same-box A/B: GPU tests on the current library (unless NO_TESTS), then the
# headline-only bench alternating the current library and MVS_LIB variants
# named in VARIANTS (libmvs_amd_<v>.so), then tools/pack_time.py.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-ab}
D=simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -60; exit $rc; }
fi
B="--no-stage --no-ring --secondary-wid 0 --steps 100 --no-cpu-baseline ${BENCH_ARGS}"
: > gpurun_out/${T}_ab.log
for rep in 1 2; do
  for v in cur ${VARIANTS}; do
    if [ $v = cur ]; then L=$PWD/$D/libmvs_amd.so; else L=$PWD/$D/libmvs_amd_$v.so; fi
    MVS_LIB=$L timeout -k 10 200 python bench.py $B > gpurun_out/${T}_b.json 2>gpurun_out/${T}_b.err || { tail -5 gpurun_out/${T}_b.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_b.json').read().strip().splitlines()[-1])
print('$v rep $rep: %.3f G cand/s  step %.1f us  kernel %.1f us  pack %.1f us' % (d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['exchange']['pack_us']))" | tee -a gpurun_out/${T}_ab.log
  done
done
[ -n "$NO_PACK" ] || timeout -k 10 200 python tools/pack_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_pack.log

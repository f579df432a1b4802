#!/bin/bash
# Round-4 iteration: GPU tests (optionally -k $PYTEST_K), then the headline-only
# bench with the tables scorer (k_score_tab) and the in-kernel-moments scorer
# (MVS_SCORE_KERNEL=mma, k_score_mma) alternating on one box.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r4}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && grep -B5 -A40 "FAILED\|Error\|error" gpurun_out/${T}_pytest.log | head -80
  # an assertion failure still lets the bench run; a crash or a time-out does not
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
B="--no-stage --no-ring --secondary-wid 0 --steps 100 --no-cpu-baseline ${BENCH_ARGS}"
: > gpurun_out/${T}_ab.log
for rep in 1 2; do
  for v in tab $([ -z "$SKIP_MMA" ] && echo mma) ${VARIANTS}; do
    KM=; L=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd.so
    if [ $v = mma ]; then KM=mma; elif [ $v != tab ]; then L=${L%.so}_$v.so; fi
    MVS_LIB=$L MVS_SCORE_KERNEL=$KM timeout -k 10 200 python bench.py $B > gpurun_out/${T}_b_$v.json 2>gpurun_out/${T}_b.err || { tail -5 gpurun_out/${T}_b.err; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_b_$v.json').read().strip().splitlines()[-1])
print('$v rep $rep: %.3f G cand/s  step %.1f us  kernel %.1f us (%s)  pack %.1f us' % (d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['kernel'], d['exchange']['pack_us']))" | tee -a gpurun_out/${T}_ab.log
  done
done
if [ -n "$PROF" ]; then
  # kernel averages of the headline (main library): k_bin, the scorer, k_score_fix, the pack
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profq_$T -o run --output-format csv -- python bench.py $B > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 1; }
  cp gpurun_out/profq_$T/run_kernel_stats.csv gpurun_out/kernel_stats_$T.csv && rm -rf gpurun_out/profq_$T
  python -c "
import csv
for r in csv.DictReader(open('gpurun_out/kernel_stats_$T.csv')):
    print('%-60s %6s %9.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))" | head -12
fi
if [ -z "$NO_STAMPS" ] && [ -f simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd_stamps.so ]; then
  timeout -k 10 200 python tools/stamps_tab.py 5 > gpurun_out/${T}_stamps.log 2>&1 || { tail -5 gpurun_out/${T}_stamps.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_stamps.log
fi

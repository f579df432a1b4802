#!/bin/bash
# Round-5 iteration: GPU tests, the headline-only bench (twice), the default
# full bench line (overlap proxy in the multi-GPU layout), bin_atomics, and a
# rocprof kernel trace of the headline (teardown crash-safe: the masked
# streams are destroyed before exit).  TAG names the outputs.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r5d}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; grep "pack_accepted (" gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; [ $rc -ne 1 ] && exit $rc; fi
fi
B="--no-stage --no-ring --secondary-wid 0 --steps 100 --no-cpu-baseline --no-overlap ${BENCH_ARGS}"
L0=$PWD/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd/libmvs_amd.so
for rep in 1 2; do
  for v in main ${VARIANTS}; do
    L=$L0; [ $v != main ] && L=${L0%.so}_$v.so
    MVS_LIB=$L timeout -k 10 300 python bench.py $B > gpurun_out/${T}_b_$v$rep.json 2>gpurun_out/${T}_b.err || { tail -5 gpurun_out/${T}_b.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/${T}_b_$v$rep.json').read().strip().splitlines()[-1])
sb=d['scaling_baseline']
print('$v rep $rep: %.3f G cand/s  step %.1f us  kernel %.1f us  pack %.1f us  with-pack step %.1f us (%s)' % (d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['exchange']['pack_us'], sb['step_ms_with_pack']*1e3, sb['layout']))" | tee -a gpurun_out/${T}_ab.log
  done
done
if [ -z "$NO_UBENCH" ]; then
  timeout -k 10 120 tools/ubench/bin_atomics > gpurun_out/${T}_bin_atomics.log 2>&1 || { cat gpurun_out/${T}_bin_atomics.log; exit 1; }
  cat gpurun_out/${T}_bin_atomics.log
fi
# rocprof kernel stats of the main library (PROF_VARIANTS=1: of every variant, twice)
PV=main; PR=1; [ -n "$PROF_VARIANTS" ] && { PV="main ${VARIANTS}"; PR="1 2"; }
for rep in $PR; do
for v in $PV; do
L=$L0; [ $v != main ] && L=${L0%.so}_$v.so
S=$T; [ $v != main ] && S=${T}_$v
MVS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$S -o run --output-format csv -- python bench.py $B > gpurun_out/${S}_prof.log 2>&1 || { tail -5 gpurun_out/${S}_prof.log; exit 1; }
f=$(find gpurun_out/prof_$S -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/${S}_kernel_stats.csv
f=$(find gpurun_out/prof_$S -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/${S}_kernel_trace.csv; rm -rf gpurun_out/prof_$S
echo "== $v (rocprof, rep $rep)"
python -c "
import csv
for r in csv.DictReader(open('gpurun_out/${S}_kernel_stats.csv')):
    print('%-60s %6s %9.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))" | head -8 | tee -a gpurun_out/${T}_ab.log
done
done
for lay in ${LAYOUTS-mask grid}; do
timeout -k 10 600 python -u bench.py --no-stage --no-ring --no-cpu-baseline --secondary-wid 0 --comm-layout $lay > gpurun_out/${T}_bench_$lay.log 2>&1 || { tail -5 gpurun_out/${T}_bench_$lay.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/${T}_bench_$lay.log').read().strip().splitlines()[-1])
print('$lay', json.dumps(d['exchange'].get('overlap_proxy'))); print(json.dumps(d['scaling_baseline']))"
done

#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "view_count or rproj" --timeout 120 > gpurun_out/pytest_rq.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_rq.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ringq.log 2>&1; rc=$?
python -c "import json; d=json.loads(open('gpurun_out/bench_ringq.log').read().strip().splitlines()[-1]); print('ring256', d['value']/1e6, 'M cand/s', d['roofline']['kernel_ms'], d['secondary'])"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ringq -o run --output-format csv -- python bench.py --scene ring256 --steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 > gpurun_out/pmc_ringq.log 2>&1; rc=$?
python - <<'PY'
import csv, collections, glob
acc = collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmc_ringq/run_counter_collection.csv'):
    for row in csv.DictReader(open(f)):
        if 'tiledg' in row['Kernel_Name']:
            acc[row['Dispatch_Id']].append(float(row['Counter_Value']))
v = [sum(x) for x in acc.values()]
print('tiledg FETCH_SIZE per launch (KiB, uncorrected):', sum(v) / max(len(v), 1))
PY
exit $rc

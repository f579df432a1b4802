#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/pytest_full.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_full.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ring.log 2>&1; rc=$?
python -c "import json; d=json.loads(open('gpurun_out/bench_ring.log').read().strip().splitlines()[-1]); print('ring256', d['value']/1e6, 'M cand/s', d['roofline']['kernel_ms'], d['secondary'])"; exit $rc

#!/bin/bash
# A/B variants (wid 5 and 3) + view-count parity tests + ring256 quick bench
export TMPDIR=/tmp
mkdir -p gpurun_out
V="${1:-0 11}"
bash tools/gpu_ab.sh "$V" 5 || exit 1
bash tools/gpu_ab.sh "$V" 3 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "view_count or score" --timeout 120 > gpurun_out/pytest_ab2.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_ab2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab2_ring.log 2>&1; rc=$?
python -c "import json; d=json.loads(open('gpurun_out/bench_ab2_ring.log').read().strip().splitlines()[-1]); print('ring256', d['value']/1e6, 'M cand/s', d['roofline']['kernel_ms'], d['secondary'])"; exit $rc

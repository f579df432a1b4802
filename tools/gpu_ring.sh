#!/bin/bash
# V > 64 path: parity tests, then the ring256 bench (tiled view groups vs direct) + rocprof stats.
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ring}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG}_tiled.log 2>&1
rc=$?; echo "bench tiled rc=$rc"; tail -1 gpurun_out/bench_${TAG}_tiled.log | cut -c1-200; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_${TAG}_tiled.log; exit $rc; }
python -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_tiled.log').read().strip().splitlines()[-1]); print(d['value']/1e6, 'M cand/s', d['roofline'], d['secondary'])"
timeout -k 10 300 python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline --kernel direct --secondary-wid 0 > gpurun_out/bench_${TAG}_direct.log 2>&1
rc=$?; echo "bench direct rc=$rc"; python -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_direct.log').read().strip().splitlines()[-1]); print(d['value']/1e6, 'M cand/s', d['roofline']['kernel_ms'])"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --scene ring256 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; cut -c1-150 gpurun_out/prof_$TAG/run_kernel_stats.csv | head -9; exit $rc

# parity tests (tiled kernel variants) + A/B + short bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q.log; [ $rc -ne 0 ] && exit $rc
AB_WID=5 timeout -k 10 300 python tools/ab_variants.py ${1:-0} > gpurun_out/ab_q.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_q.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-sample 20000 > gpurun_out/bench_q.log 2>&1; rc=$?; tail -1 gpurun_out/bench_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']/1e9, d['roofline']['kernel_ms'], d['secondary'])"; exit $rc

#!/bin/bash
# Round-end set on one box: GPU tests, smoke(), the default bench line (its
# roofline from the newest profiles/rNN/pmc.json), then the N=2 exchange rehearsal
# (two ranks on cuda:0 over gloo).  TAG names the outputs.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-fin}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_full.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_bench_full.log | cut -c1-300
bash tools/gpu_rehearse_multi.sh

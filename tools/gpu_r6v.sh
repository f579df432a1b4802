#!/bin/bash
# Round 6, last session: the paired-scorer probe (one stream / two contexts
# free / two contexts gated by mvs_pair_scorers), then the round-end set.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for m in gate ctx gate; do
  MODE=$m timeout -k 10 180 python tools/pipeline_probe.py 200 >> gpurun_out/r6v_probe.log 2>&1 || { tail -20 gpurun_out/r6v_probe.log; exit 1; }
done
grep mode gpurun_out/r6v_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -x -v --timeout 120 --timeout-method thread -k paired > gpurun_out/r6v_pair_test.log 2>&1 || { tail -30 gpurun_out/r6v_pair_test.log; exit 1; }
tail -1 gpurun_out/r6v_pair_test.log
bash tools/gpu_round_end.sh

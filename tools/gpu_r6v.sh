#!/bin/bash
# Round 6, last session: the paired-scorer probe (two contexts gated by
# mvs_pair_scorers / two contexts free), its parity test, the headline-only
# bench with --pipeline 0 / 1 (twice each), then the round-end set.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for m in gate ctx; do
  MODE=$m timeout -k 10 180 python tools/pipeline_probe.py 200 >> gpurun_out/r6v_probe.log 2>&1 || { tail -20 gpurun_out/r6v_probe.log; exit 1; }
done
grep mode gpurun_out/r6v_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -x -v --timeout 120 --timeout-method thread -k paired > gpurun_out/r6v_pair_test.log 2>&1 || { tail -30 gpurun_out/r6v_pair_test.log; exit 1; }
tail -1 gpurun_out/r6v_pair_test.log
B="--no-stage --no-ring --secondary-wid 0 --steps 100 --no-cpu-baseline --no-overlap"
for rep in 1 2; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py $B --pipeline $p > gpurun_out/r6v_b_p$p$rep.json 2>gpurun_out/r6v_b.err || { tail -5 gpurun_out/r6v_b.err; exit 1; }
    python tools/ab_line.py gpurun_out/r6v_b_p$p$rep.json "pipeline $p rep $rep" | tee -a gpurun_out/r6v_ab.log
  done
done
[ -n "$NO_RE" ] && exit 0
bash tools/gpu_round_end.sh

#!/bin/bash
# Headline-only bench at several scorer grids (MVS_SCORER_WGS), twice each,
# same box.  Usage (GPU box): GRIDS="0 480" bash tools/grid_ab.sh TAG
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${1:-grid}
B="--no-stage --no-ring --secondary-wid 0 --steps 100 --no-cpu-baseline --no-overlap"
for rep in 1 2; do
  for g in ${GRIDS:-0 480}; do
    MVS_SCORER_WGS=$g timeout -k 10 300 python bench.py $B > gpurun_out/${T}_$g.json 2>gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/${T}_$g.json').read().strip().splitlines()[-1])
print('grid $g rep $rep: %.3f G cand/s  step %.1f us  kernel %.1f us' % (d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3))" | tee -a gpurun_out/${T}_ab.log
  done
done

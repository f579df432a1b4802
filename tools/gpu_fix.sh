#!/bin/bash
# Guard-band re-score: how many lanes take the exact path on the bench batch, and k_score_fix's per-call time.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/fix_count.py > gpurun_out/fix_count.log 2>&1 || { tail -5 gpurun_out/fix_count.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fix_count.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fixprof -o run --output-format csv -- python tools/ab_variants.py 0 > gpurun_out/fixprof.log 2>&1 || { tail -5 gpurun_out/fixprof.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/fixprof/**/*kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if 'k_score_fix' in k or 'k_bin' in k or 'k_scatter' in k or 'k_tile_scan' in k or 'tiled3' in k:
        d[k[:60]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    print(k, ' '.join('%.1f' % x for x in v))
PY

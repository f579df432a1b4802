#!/bin/bash
# Kernel iteration: scorer parity subset, stamps A/B (old vs new stamps libs),
# headline rocprof kernel stats.  TAG names the outputs.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-it}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-score or sweep or view or mask or wide or ncc or stage_vs or mypatch or exact}" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/${T}_pytest.log | head -60; exit $rc; }
if [ -z "$NO_STAMPS" ]; then TAG=$T bash tools/gpu_stamps_ab.sh || exit 1; fi
B="--no-stage --no-ring --secondary-wid 0 --steps 50 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py $B > gpurun_out/${T}_prof.log 2>&1 || exit $?
find gpurun_out/${T}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_kernel_stats.csv \;
rm -rf gpurun_out/${T}_prof
python3 - <<'PY'
import csv, os
T = os.environ.get("TAG", "it")
for r in csv.DictReader(open(f"gpurun_out/{T}_kernel_stats.csv")):
    if "at::" in r["Name"]: continue
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1000:8.2f} us")
PY
grep -o '"value": [0-9.e+]*' gpurun_out/${T}_prof.log | head -1

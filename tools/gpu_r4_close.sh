#!/bin/bash
# Round-4 closing call in one box session (the pool gives few boxes): GPU
# tests + smoke (tools/gpu_final_r4.sh), a same-box A/B of the library
# against $VARIANTS (headline only), then PMC passes, rocprof stats and the
# default bench line (tools/gpu_final_r4.sh without its tests).
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r4z}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
NO_TESTS=1 NO_STAMPS=${NO_STAMPS} SKIP_MMA=1 TAG=${T}ab bash tools/gpu_r4.sh || exit $?
NO_TESTS=1 TAG=$T bash tools/gpu_final_r4.sh || exit $?

#!/bin/bash
# Round-5 probes: k_bin's ranking by counter layout (ubench/bin_atomics), the
# overlap probe with the unrolled proxy copy under CU masks and with the pack
# on the comm stream, and a kernel trace of one variant.
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
T=${TAG:-r5b}
[ -z "$FROM_C" ] && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "pack or exchange or bench_ranks or records" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; [ -z "$FROM_C" ] && { tail -2 gpurun_out/${T}_pytest.log; grep "pack_accepted (" gpurun_out/${T}_pytest.log; }; [ -z "$FROM_C" ] && [ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/${T}_pytest.log | head -80; exit $rc; }
timeout -k 10 120 tools/ubench/bin_atomics > gpurun_out/${T}_bin_atomics.log 2>&1 || { cat gpurun_out/${T}_bin_atomics.log; exit 1; }
cat gpurun_out/${T}_bin_atomics.log
for args in "base cumask pipe cumask+pipe --free 16" "cumask cumask+pipe --free 32" "cumask cumask+pipe --free 16 --mask-order spread" "cumask --free 16 --mask-order lo"; do
  echo "== $args"
  timeout -k 10 300 python -u tools/overlap_probe.py $args > gpurun_out/${T}_probe.log 2>&1 || { tail -20 gpurun_out/${T}_probe.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_probe.log
done
for v in "cumask+pipe" "base"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_$T -o run --output-format csv -- python tools/overlap_probe.py $v --free 16 --steps 8 > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
  f=$(find gpurun_out/trace_$T -name '*kernel_trace.csv' | head -1)
  cp "$f" gpurun_out/${T}_${v}_kernel_trace.csv && rm -rf gpurun_out/trace_$T
  python tools/overlap_timeline.py gpurun_out/${T}_${v}_kernel_trace.csv 60 45 > gpurun_out/${T}_${v}_timeline.txt
  echo "== trace $v"; cat gpurun_out/${T}_${v}_timeline.txt | cut -c1-110
done
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1; grep -E "^\s*(TA_|TD_|TCP_)" gpurun_out/${T}_counters.txt | head -80 > gpurun_out/${T}_counters_ta.txt; wc -l gpurun_out/${T}_counters.txt

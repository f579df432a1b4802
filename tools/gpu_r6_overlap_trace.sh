export TMPDIR=/tmp
cd /root/repo
mkdir -p gpurun_out
# 1. the overlap proxy under a kernel trace (one variant: torch streams, grid 512)
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r6i_tr -o run --output-format csv -- python tools/overlap_probe.py base --steps 30 > gpurun_out/r6i_probe.log 2>&1
rc=$?; tail -4 gpurun_out/r6i_probe.log; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/r6i_tr -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/r6i_kernel_trace.csv; rm -rf gpurun_out/r6i_tr
# 2. the masked layout under rocprofv3 (round 5's exit SIGSEGV): the bench's
#    masked streams are left to the atexit hook here? no: bench closes them;
#    run it as the bench does, and a script that does not close them
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6i_mask -o run --output-format csv -- python bench.py --comm-layout mask --pack-on-comm --no-stage --no-ring --no-cpu-baseline --secondary-wid 0 --steps 30 > gpurun_out/r6i_mask.log 2>&1
echo "masked-layout bench under rocprofv3: rc=$?"; grep -c SIGSEGV gpurun_out/r6i_mask.log
rm -rf gpurun_out/r6i_mask

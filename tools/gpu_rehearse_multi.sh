#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks on cuda:0 over gloo
# (RCCL refuses two ranks on one device); checks the exchange code path runs.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --secondary-wid 0 > gpurun_out/bench_rehearse2.log 2>&1
rc=$?; echo "rehearse rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_rehearse2.log | tail -3 | cut -c1-600; exit $rc

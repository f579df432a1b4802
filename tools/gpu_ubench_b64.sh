#!/bin/bash
# LDS read-shape cost microbenchmark (tools/ubench/lds_b64.hip)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/lds_b64 > gpurun_out/lds_b64.log 2>&1; rc=$?; cat gpurun_out/lds_b64.log; exit $rc

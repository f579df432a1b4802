#!/bin/bash
# LDS 16-byte read alignment / cost microbenchmark (tools/ubench/lds_b128.hip)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/lds_b128 > gpurun_out/lds_b128.log 2>&1; rc=$?; cat gpurun_out/lds_b128.log; exit $rc

#!/bin/bash
# SURVEY.md section 5 sanitizer build: the CPU test suite with the oracle
# (oracle/libmvs_oracle_asan.so, make -C oracle asan) and the library's host
# code (libmvs_amd_asan.so, build_lib.py --asan) under ASan + UBSan (clang
# runtime, preloaded into the Python process; no GPU needed, CPU container
# only: the GPU pool runs no sanitizers on device code).  Log:
# profiles/r03/asan_cpu.log.
cd "$(dirname "$0")/.." || exit 1
PKG=simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd
make -s -C oracle asan || exit 1
python $PKG/build_lib.py --asan > /dev/null || exit 1
RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
mkdir -p profiles/r03
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
MVS_ORACLE_LIB=$PWD/oracle/libmvs_oracle_asan.so MVS_LIB=$PWD/$PKG/libmvs_amd_asan.so \
  timeout -k 10 1800 python -m pytest tests -m "not gpu" -v -p no:cacheprovider > profiles/r03/asan_cpu.log 2>&1
rc=$?
grep -c "ERROR: AddressSanitizer\|runtime error:" profiles/r03/asan_cpu.log
tail -3 profiles/r03/asan_cpu.log
exit $rc

export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $@; do MVS_VARIANT=$v timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_v$v.log 2>&1; rc=$?; echo "== variant $v"; tail -6 gpurun_out/stamps_v$v.log; [ $rc -ne 0 ] && exit $rc; done
exit 0

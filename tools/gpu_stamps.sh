export TMPDIR=/tmp
mkdir -p gpurun_out
MVS_VARIANT=6 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps6.log 2>&1; rc=$?; tail -6 gpurun_out/stamps6.log; [ $rc -ne 0 ] && exit $rc
MVS_VARIANT=0 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps0.log 2>&1; rc=$?; tail -6 gpurun_out/stamps0.log; [ $rc -ne 0 ] && exit $rc
export MVS_VARIANT=6
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_MFMA_I8 SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_m6/p$i -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --secondary-wid 0 > gpurun_out/pmc_m6_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_m6_p$i.log; exit $rc; }
done
exit 0

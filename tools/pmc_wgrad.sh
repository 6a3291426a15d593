cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in new old; do
  if [ $v = old ]; then export MSU_WGRAD_GENERIC=1; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc_$v -o p1 --output-format csv -- python3 $R/tools/wgrad_one.py 524288 96 96 10 > $R/gpurun_out/pmc_$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d $R/gpurun_out/pmc_$v -o p2 --output-format csv -- python3 $R/tools/wgrad_one.py 524288 96 96 10 >> $R/gpurun_out/pmc_$v.log 2>&1 || exit 1
done
echo done

cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc_conv -o p1 --output-format csv -- python3 $R/tools/conv_one.py 0 3 > $R/gpurun_out/pmc_conv.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $R/gpurun_out/pmc_conv -o p2 --output-format csv -- python3 $R/tools/conv_one.py 0 3 >> $R/gpurun_out/pmc_conv.log 2>&1 || exit 1
echo done

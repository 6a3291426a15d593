# SQ counter passes over any command: bash tools/pmc_generic.sh NAME FILTER cmd...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NAME=$1; FLT=$2; shift 2
O=$R/gpurun_out/pmcg_$NAME
mkdir -p $O
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" \
            "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "GRBM_GUI_ACTIVE TCC_HIT TCC_MISS TCC_BUSY TA_BUSY" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctrs -d $O -o p$i --output-format csv -- "$@" > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
for f in $O/p*_counter_collection.csv; do python3 $R/tools/pmc_sum.py $FLT $f; done

# Counter passes over one token-GEMM shape: bash tools/pmc_tok.sh M N K [epi]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_tok_$1_$2_$3
mkdir -p $O
run() { timeout -s KILL 60 rocprofv3 --pmc $2 -d $O -o $1 --output-format csv -- python3 $R/tools/tok_one.py $ARGS > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }; }
ARGS="$1 $2 $3 ${4:-0} 3"
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
run sq2 "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VALU"
for f in $O/*_counter_collection.csv; do python3 $R/tools/pmc_sum.py tokgemm $f; done

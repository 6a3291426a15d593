# Counter passes over one window-attention shape (fwd + bwd):
#   bash tools/pmc_attn.sh TAG res nh shift [p_drop]   (stage 0 of the 1024^2 bench: 256 3 0)
#   bash tools/pmc_attn.sh TAG fused [p_drop]           (the fused stage-0 unit, tools/attn_qkv_one.py)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/pmc_attn_$TAG
mkdir -p $O
if [ "$1" = fused ]; then PROG=attn_qkv_one.py; ARGS="3 ${2:-0.05}"; KERNS="attn_qkv_fwd attn_bwd"
else PROG=attn_one.py; ARGS="$1 $2 $3 1 3 ${4:-0.0}"; KERNS="attn_fwd attn_bwd"; fi
run() { timeout -s KILL 60 rocprofv3 --pmc $2 -d $O -o $1 --output-format csv -- python3 $R/tools/$PROG $ARGS > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
run sq2 "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VALU"
run sq3 "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/tools/$PROG $ARGS > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
# LDS-array cycles (the bank-conflict ratio's denominator); not fatal if the counter is absent
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE -d $O -o sq4 --output-format csv -- python3 $R/tools/$PROG $ARGS > $O/sq4.log 2>&1 || tail -3 $O/sq4.log
for k in $KERNS; do echo "== $k"; for f in $O/*_counter_collection.csv; do python3 $R/tools/pmc_sum.py $k $f; done; done
grep -h attn $O/kt_kernel_stats.csv | cut -c1-200

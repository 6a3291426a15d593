# SQ counter passes over the refine conv (v3 forward as the model runs it, then the backward:
# v3 dgrad + v2 wgrad), plus a kernel trace:   bash tools/pmc_conv3.sh TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1
O=$R/gpurun_out/pmc_conv3_$TAG
mkdir -p $O
run() {  # name "counters" args...
  local n=$1 c=$2; shift 2
  timeout -s KILL 60 rocprofv3 --pmc $c -d $O -o $n --output-format csv -- python3 $R/tools/conv_one.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
}
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
S2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"
S3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
for mode in fwd bwd; do
  a="0 3 $mode act"
  [ $mode = bwd ] && a="0 3 bwd"
  run ${mode}_sq1 "$S1" $a
  run ${mode}_sq2 "$S2" $a
  run ${mode}_sq3 "$S3" $a
  timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $O -o ${mode}_kt --output-format csv -- python3 $R/tools/conv_one.py $a > $O/${mode}_kt.log 2>&1 || { tail -5 $O/${mode}_kt.log; exit 1; }
done
for mk in fwd:conv3x3_v${CONV_V:-4} bwd:conv3x3_v${CONV_V:-4} bwd:conv3x3_wgrad_v2; do
  m=${mk%%:*}; k=${mk#*:}
  echo "== $m $k"
  for f in $O/${m}_sq?_counter_collection.csv; do python3 $R/tools/pmc_sum.py $k $f; done
done
grep -h conv3x3 $O/*_kt_kernel_stats.csv | cut -c1-200
echo done

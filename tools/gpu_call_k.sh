# standalone kernel timings: streaming reference, LayerNorm, weight-gradient plans (K split on
# / off), refine convs (halo spread on / off), window attention
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-k1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/${TAG}_$n.log 2>&1
  local rc=$?
  grep -v amdgpu.ids $O/${TAG}_$n.log | tail -20
  if [ $rc -ne 0 ]; then echo "$n rc=$rc"; exit $rc; fi
}
run stream 120 python -u $R/tools/kbench.py stream
run ln 180 python -u $R/tools/kbench.py ln
run lnadd 180 python -u $R/tools/kbench.py lnadd
run wgrad_wk1 180 env KB_STAGE=0 MSU_WGRAD_WK=1 python -u $R/tools/kbench.py wgrad
run wgrad_wk0 180 env KB_STAGE=0 MSU_WGRAD_WK=0 python -u $R/tools/kbench.py wgrad
run wgrad1_wk1 180 env KB_STAGE=1 MSU_WGRAD_WK=1 python -u $R/tools/kbench.py wgrad
run wgrad1_wk0 180 env KB_STAGE=1 MSU_WGRAD_WK=0 python -u $R/tools/kbench.py wgrad
run conv_hs0 240 env MSU_CONV_HALO=0 python -u $R/tools/kbench.py conv
run conv_hs1 240 env MSU_CONV_HALO=1 python -u $R/tools/kbench.py conv
[ -f $R/tools/exp/libmsunet_noslp_conv.so ] && run conv_noslp 240 env MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_noslp_conv.so python -u $R/tools/kbench.py conv
run attn 240 python -u $R/tools/kbench.py attn
[ -f $R/tools/exp/libmsunet_noslp_attn.so ] && run attn_noslp 240 env MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_noslp_attn.so python -u $R/tools/kbench.py attn
echo done

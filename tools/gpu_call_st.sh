# GPU op tests, then same-box A/Bs of the round-3 switches (transposed weight shadow, wgrad
# K-split plans, v3 halo spread, LayerNorm rows in flight)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest $R/tests/test_gpu_shadow_t.py $R/tests/test_gpu_ops.py \
  -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/st_tests.log 2>&1
rc=$?; tail -5 $O/st_tests.log; [ $rc -ne 0 ] && exit $rc
bash $R/tools/gpu_ab.sh st "MSU_SHADOW_T=1" "MSU_SHADOW_T=0" 2 || exit 1
bash $R/tools/gpu_ab.sh wk "MSU_WGRAD_WK=1" "MSU_WGRAD_WK=0" 2 || exit 1
bash $R/tools/gpu_ab.sh hs "MSU_CONV_HALO=0" "MSU_CONV_HALO=1" 2 || exit 1
bash $R/tools/gpu_ab.sh nr "MSU_LN_NR=2" "MSU_LN_NR=1" 2 || exit 1
echo done

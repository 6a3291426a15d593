# transposed weight shadow, wgrad K-split plans, v3 halo spread, attention padded-key skip:
# GPU op tests, same-box A/Bs, then the conv SQ counters
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
bash $R/tools/pmc_conv3.sh c3a > $O/pmc_conv3_c3a.txt 2>&1
rc=$?; tail -70 $O/pmc_conv3_c3a.txt; exit $rc

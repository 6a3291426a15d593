# r03l: RCCL child-process tests, conv v4 parity + timing (v4 vs v3), conv PMC, GEMM tables
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -m gpu -q -k "conv" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03l_conv_tests.log 2>&1; rc=$?; echo "conv tests rc=$rc"; tail -2 $O/r03l_conv_tests.log; [ $rc -gt 1 ] && exit $rc
for v in 4 3 4 3; do echo "== v$v"; MSU_CONV_V=$v timeout -k 10 120 python3 -u $R/tools/kbench.py conv 2>&1 | grep -v "Warn\|amdgpu.ids" || exit 1; done > $O/r03l_conv_ab.log
cat $O/r03l_conv_ab.log
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_rccl.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r03l_rccl.log 2>&1; rc=$?; echo "rccl rc=$rc"; tail -2 $O/r03l_rccl.log; [ $rc -gt 1 ] && exit $rc
bash $R/tools/pmc_conv3.sh r03l > $O/r03l_pmc_conv3.log 2>&1; echo "pmc rc=$?"
timeout -k 10 300 python3 -u $R/tools/kbench.py nt > $O/r03l_nt.log 2>&1 || exit 1
timeout -k 10 300 python3 -u $R/tools/kbench.py tok > $O/r03l_tok.log 2>&1 || exit 1
echo done

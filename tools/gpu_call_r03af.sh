# r03af: one-pass Linear backward with compiler-tracked staging loads (issued on every path, D = 3 / 2):
# parity, microbench, bench A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_linbwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03af_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/r03af_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py > $O/r03af_linbwd.log 2>&1 || exit 1
grep "linbwd" $O/r03af_linbwd.log
bash $R/tools/gpu_bench_ab.sh r03af "" "MSU_LINBWD=0" "" "MSU_LINBWD=0"

# r03ah: one-pass Linear backward with 16 x 16 input-gradient tiles over all waves for K = 96:
# parity, microbench, bench A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_linbwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03ah_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/r03ah_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py > $O/r03ah_linbwd.log 2>&1 || exit 1
grep "linbwd" $O/r03ah_linbwd.log
bash $R/tools/gpu_bench_ab.sh r03ah "" "MSU_LINBWD=0" "" "MSU_LINBWD=0"

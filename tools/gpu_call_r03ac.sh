# r03ac: one-pass Linear backward v5 (saddr loads, tr-conflict-free X, spread bias): parity, microbench, bench A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_linbwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03ac_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 $O/r03ac_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u $R/tools/linbwd_bench.py > $O/r03ac_linbwd.log 2>&1 || exit 1
grep linbwd $O/r03ac_linbwd.log
bash $R/tools/gpu_bench_ab.sh r03ac "MSU_LINBWD=1" "" "MSU_LINBWD=1" ""

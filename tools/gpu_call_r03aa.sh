# r03aa: one-pass Linear backward v3 (untracked staging loads, counted waits): parity, microbench, bench A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_linbwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03aa_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 $O/r03aa_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u $R/tools/linbwd_bench.py > $O/r03aa_linbwd.log 2>&1 || exit 1
grep linbwd $O/r03aa_linbwd.log
bash $R/tools/gpu_bench_ab.sh r03aa "" "MSU_LINBWD=0" "" "MSU_LINBWD=0"

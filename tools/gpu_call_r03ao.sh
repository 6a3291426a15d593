# r03ao: one-pass Linear backward with 64-token steps for qkv / proj (build with MSU_LB_TS64=1 in
# tools/exp): parity through that build, microbench vs the 32-token default, bench A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
X64=$R/tools/exp/libmsunet_gemm_linbwd_ts64.so
MSU_LIB_OVERRIDE=$X64 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_linbwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03ao_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/r03ao_tests.log; [ $rc -ne 0 ] && exit $rc
L=$O/r03ao_linbwd.log; : > $L
for rep in 1 2; do
  for v in ts64 ts32; do
    echo "== $v" >> $L
    if [ $v = ts64 ]; then export MSU_LIB_OVERRIDE=$X64; else unset MSU_LIB_OVERRIDE; fi
    timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py 96 288 >> $L 2>&1 || exit 1
    timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py 96 96 >> $L 2>&1 || exit 1
  done
done
unset MSU_LIB_OVERRIDE
grep "==\|linbwd" $L | sed 's/dgrad.*//'
bash $R/tools/gpu_bench_ab.sh r03ao "MSU_LIB_OVERRIDE=$X64" "" "MSU_LIB_OVERRIDE=$X64" ""

# r03x: one-pass stage-0 Linear backward: parity tests, then same-box bench A/B (on / off)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_linbwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03x_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 $O/r03x_tests.log; [ $rc -ne 0 ] && exit $rc
bash $R/tools/gpu_bench_ab.sh r03x "" "MSU_LINBWD=0" "" "MSU_LINBWD=0" "MSU_WGRAD_TARGET_S23=128" "MSU_WGRAD_TARGET_S23=512"

# r03t: NT / token GEMM wait-count fix -> eager determinism matrix, GEMM parity tests, bench
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_nt_gemm.py $R/tests/test_gpu_tok_gemm.py $R/tests/test_gpu_graph.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/r03t_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/r03t_tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python3 -u $R/tools/determinism_matrix.py 8 > $O/r03t_determinism.log 2>&1; echo "det rc=$?"; grep "side=" $O/r03t_determinism.log
bash $R/tools/gpu_bench_ab.sh r03t "" ""

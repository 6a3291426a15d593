# r03r: how much the side stream costs the main stream (ablations, wrong results by design),
# NT GEMM static priority, attention backward without row loads (ablation lib)
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_bench_ab.sh r03r "" "MSU_EXP_SKIP_WGRAD=1" "--skip-dead" "MSU_NT_PRIO=1" "" "MSU_NT_PRIO=1" || exit 1
bash $R/tools/exp_run.sh attn window_attention_mfma 4 > $R/gpurun_out/r03r_attn_exp.log 2>&1; echo "exp rc=$?"
grep "stage0" $R/gpurun_out/r03r_attn_exp.log
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_rccl.py $R/tests/test_gpu_graph.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/r03r_rccl.log 2>&1; echo "rccl rc=$?"; tail -3 $R/gpurun_out/r03r_rccl.log

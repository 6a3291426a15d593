# One GPU call, named steps run in order, each under its own time limit; the call stops at the
# first step that faults, aborts or times out (exit status > 1).  Logs: gpurun_out/TAG_<step>.log
#   bash tools/gpu_call.sh TAG step [step ...]
# steps: tests_new (the round's new GPU tests), tests (whole -m gpu suite), smoke, bench,
#        prof (eager step under rocprofv3 --kernel-trace --stats), conv_pmc (refine-conv HBM
#        counters), attn_pmc, gemm_mem (NT GEMM / weight-gradient memory counters), kern (kernel
#        timings of the GEMM families), ab_* (same-box bench A/Bs, see the case list)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $secs "$@" > $O/${TAG}_$name.log 2>&1
  local rc=$?
  tail -4 $O/${TAG}_$name.log
  echo "== $name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
  case $s in
    tests_new) step tests_new 900 $PYT -m gpu $R/tests/test_gpu_handoff.py $R/tests/test_gpu_mlp_infer.py \
                 $R/tests/test_gpu_model.py $R/tests/test_gpu_ln_side.py ;;
    linbwd) step linbwd 600 $PYT -m gpu $R/tests/test_gpu_linbwd.py $R/tests/test_gpu_ln_side.py $R/tests/test_gpu_handoff.py ;;
    aten) step aten 600 $PYT -m gpu $R/tests/test_gpu_ops.py -k 'conv_wgrad or conv_weight or refine_conv' $R/tests/test_gpu_ln_side.py $R/tests/test_gpu_trainer.py $R/tests/test_gpu_mlp_infer.py ;;
    trainer) step trainer 900 $PYT -m gpu $R/tests/test_gpu_trainer.py $R/tests/test_gpu_graph.py $R/tests/test_gpu_rccl.py $R/tests/test_gpu_baseline_shapes.py $R/tests/test_gpu_step_parity.py ;;
    flag) step flag 900 $PYT -m gpu $R/tests/test_gpu_trainer.py $R/tests/test_gpu_graph.py $R/tests/test_gpu_ops.py -k 'dynamic_loss or nonfinite or trainer or graph or adamw' ;;
    parity) step parity 900 $PYT -s -m gpu $R/tests/test_gpu_step_parity.py ;;
    nt_tests) step nt_tests 600 $PYT -m gpu $R/tests/test_gpu_nt_gemm.py $R/tests/test_routing.py ;;
    nt_ab) step nt_ab 300 python -u $R/tools/nt_ab.py 3 20 ;;
    nt_shapes)
      # NT GEMM kernel times per stage 1-3 shape: this build (A) vs AB_LIB (B), interleaved twice
      for L in "" "$AB_LIB" "" "$AB_LIB"; do
        MSU_LIB_OVERRIDE=$L timeout -k 10 200 python -u $R/tools/nt_shapes.py 20 ${L:+B} >> $O/${TAG}_nt_shapes.log 2>&1 || exit 3
      done
      python3 $R/tools/ab_table.py $O/${TAG}_nt_shapes.log ;;
    nt_a3)
      # the 256 x 192 NT tile on the A3W2 ring vs the two-stage ring, interleaved twice; then the NT
      # tests with A3 on
      for A in 0 1 0 1; do
        NT_A3=$A timeout -k 10 200 python -u $R/tools/nt_shapes.py 20 >> $O/${TAG}_nt_a3.log 2>&1 || exit 3
      done
      python3 $R/tools/ab_table.py $O/${TAG}_nt_a3.log F0A0 F0A1
      step nt_a3_tests 600 $PYT -m gpu $R/tests/test_gpu_nt_gemm.py ;;
    nt_dyn)
      # NT GEMM kernel times per shape: the tile queue (default) vs MSU_NT_DYN=0, interleaved twice
      for E in 1 0 1 0; do
        MSU_NT_DYN=$E timeout -k 10 200 python -u $R/tools/nt_shapes.py 20 dyn$E >> $O/${TAG}_nt_dyn.log 2>&1 || exit 3
      done
      python3 $R/tools/ab_table.py $O/${TAG}_nt_dyn.log dyn1 dyn0 ;;
    nt_force)
      # NT GEMM kernel times per shape under each forced tile form (tools/nt_shapes.py NT_FORCE)
      for F in 0 1 2 3 0 1; do
        NT_FORCE=$F timeout -k 10 200 python -u $R/tools/nt_shapes.py 20 >> $O/${TAG}_nt_force.log 2>&1 || exit 3
      done
      for F in F1 F2 F3; do python3 $R/tools/ab_table.py $O/${TAG}_nt_force.log cur $F; done ;;
    nt_exp)
      for X in 4 8; do
        echo "== MSU_EXP=$X (1: no DMA, 2: no fragment reads, 4: no MFMA, 8: no epilogue)" >> $O/${TAG}_nt_exp.log
        MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_nt_$X.so timeout -k 10 200 python -u $R/tools/nt_ab.py 1 20 >> $O/${TAG}_nt_exp.log 2>&1 || exit 3
      done
      cat $O/${TAG}_nt_exp.log ;;
    tests) step tests 1000 python -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    smoke) step smoke 300 python -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 480 python -u $R/bench.py
           grep '^{' $O/${TAG}_bench.log > $O/${TAG}_bench.json ;;
    # MSU_GRAPH=0: the profiler's per-launch host cost makes the bench's auto policy pick the
    # single-stream graph replay; the profile must show the eager step the bench line measures
    prof) MSU_GRAPH=0 step prof 420 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o p --output-format csv -- \
            python3 $R/bench.py --steps 8 --warmup 4 --no-roofline --no-cpu-baseline --no-input-pipeline ;;
    # the bench command itself under the profiler (roofline included): the roofline kernel's
    # launches in the trace against the bench line's HIP-event time
    bprof) step bprof 600 rocprofv3 --kernel-trace --stats -d $O/${TAG}_bprof -o p --output-format csv -- \
             python3 $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-input-pipeline
           grep '^{' $O/${TAG}_bprof.log > $O/${TAG}_bprof.json
           python3 $R/tools/roofline_trace.py $O/${TAG}_bprof/p_kernel_trace.csv $O/${TAG}_bprof.json > $O/${TAG}_roofline_trace.txt
           cat $O/${TAG}_roofline_trace.txt ;;
    conv_pmc)
      timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/${TAG}_pmcconv -o conv_fetch --output-format csv -- python3 $R/tools/conv_one.py 0 3 fwd act > /dev/null 2>&1 || exit 3
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/${TAG}_pmcconv -o conv_write --output-format csv -- python3 $R/tools/conv_one.py 0 3 fwd act > /dev/null 2>&1 || exit 3
      python3 $R/tools/pmc_json.py conv3x3_v3_kernel $O/${TAG}_pmcconv/conv_fetch_counter_collection.csv \
        $O/${TAG}_pmcconv/conv_write_counter_collection.csv $O/${TAG}_conv3x3_fwd_pmc.json && cat $O/${TAG}_conv3x3_fwd_pmc.json ;;
    attn_pmc) step attn_pmc 400 bash $R/tools/pmc_attn.sh $TAG 256 3 3 0.05 ;;
    fused_pmc) step fused_pmc 400 bash $R/tools/pmc_attn.sh ${TAG}_fused fused 0.05 ;;
    gemm_mem)
      # memory-side counters of the NT GEMM and the weight gradient at a stage-2 shape: HBM bytes
      # (FETCH_SIZE x2 / WRITE_SIZE) and the L2 hit rate, one counter group per pass
      for prog in "nt_one.py 32768 1152 384 10" "wgrad_one.py 32768 1152 384 10"; do
        n=${prog%%.py*}
        for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
          tagc=$(echo $c | cut -d' ' -f1)
          timeout -s KILL 90 rocprofv3 --pmc $c -d $O/${TAG}_mem_${n}_$tagc -o p --output-format csv -- python3 $R/tools/$prog > /dev/null 2>&1 || exit 3
        done
      done
      for f in $O/${TAG}_mem_nt_one_*/p_counter_collection.csv; do echo "== $f"; python3 $R/tools/pmc_sum.py gemm_nt $f; done
      for f in $O/${TAG}_mem_wgrad_one_*/p_counter_collection.csv; do echo "== $f"; python3 $R/tools/pmc_sum.py wgrad_wave $f; done ;;
    kern)
      for shp in "32768 1152 384" "8192 2304 768" "131072 576 192" "524288 288 96"; do
        timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 30 2>&1 | grep wgrad >> $O/${TAG}_kern.log || exit 3
      done
      for shp in "32768 1152 384" "32768 384 1536" "32768 1536 384" "131072 192 576" "131072 576 192" "8192 768 3072" "8192 3072 768"; do
        timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_kern.log || exit 3
      done
      cat $O/${TAG}_kern.log ;;
    gelu_tests) step gelu_tests 900 $PYT -m gpu $R/tests/test_gpu_tok_gemm.py $R/tests/test_gpu_nt_gemm.py \
                  $R/tests/test_gpu_linbwd.py $R/tests/test_gpu_ln_side.py $R/tests/test_gpu_ops.py ;;
    mlp_s1) step mlp_s1 200 python -u $R/tools/mlp_s1_one.py 20 ;;
    mlp_s1_ab)
      # stage-1 fused MLP: this build vs AB_LIB (kernel times twice each, then AB_LIB's MLP tests)
      for L in "" "$AB_LIB" "" "$AB_LIB"; do
        echo "== ${L:-cur}" >> $O/${TAG}_mlp_s1_ab.log
        MSU_LIB_OVERRIDE=$L timeout -k 10 200 python -u $R/tools/mlp_s1_one.py 20 >> $O/${TAG}_mlp_s1_ab.log 2>&1 || exit 3
      done
      cat $O/${TAG}_mlp_s1_ab.log
      MSU_LIB_OVERRIDE=$AB_LIB step mlp_tests_B 600 $PYT -m gpu $R/tests/test_gpu_mlp_infer.py ;;
    ab_mlp_s1) bash $R/tools/gpu_bench_ab.sh ${TAG}_mlps1 "" "MSU_MLP_S1=0" "" "MSU_MLP_S1=0" "" "MSU_MLP_S1=0" || exit 3 ;;
    mlp_tests) step mlp_tests 600 $PYT -m gpu $R/tests/test_gpu_mlp_infer.py $R/tests/test_gpu_tok_gemm.py ;;
    attn_tests) step attn_tests 900 $PYT -m gpu $R/tests/test_gpu_attn_qkv.py $R/tests/test_gpu_production_parity.py \
                  $R/tests/test_gpu_ops.py -k "attn or attention or window" ;;
    attn_kern)
      # window-attention kernel times per stage shape (8 x res^2, nh heads, shift 3, dropout 0.05),
      # this build vs an override library (AB_LIB)
      for L in "" "$AB_LIB"; do
        for shp in "256 3" "128 6" "64 12" "32 24"; do
          d=$O/${TAG}_attnk_$(basename "${L:-cur}" .so)_${shp// /_}
          MSU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/attn_one.py $shp 3 1 6 0.05 > /dev/null 2>&1 || exit 3
          python3 $R/tools/kstats.py $d/p_kernel_stats.csv attn "${L:+B}${shp// /x}" >> $O/${TAG}_attn_kern.log
        done
      done
      cat $O/${TAG}_attn_kern.log ;;
    ab_conv_side) bash $R/tools/gpu_bench_ab.sh ${TAG}_convside "" "MSU_CONV_SIDE=0" "" "MSU_CONV_SIDE=0" "" "MSU_CONV_SIDE=0" || exit 3 ;;
    conv_exp)
      # refine-conv kernel times with ablation builds (tools/build_exp.sh conv3x3 64 128 256 512)
      for X in ${CONV_EXP:-0 64 128 256 512}; do
        L=""; [ $X != 0 ] && L=$R/tools/exp/libmsunet_conv3x3_$X.so
        IFS=';' read -ra CARGS <<< "${CONV_EXP_ARGS:-1 6 bwd;0 6 fwd act}"
        for args in "${CARGS[@]}"; do
          d=$O/${TAG}_convexp_${X}_${args// /_}
          MSU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/conv_one.py $args > /dev/null 2>&1 || exit 3
          python3 $R/tools/kstats.py $d/p_kernel_stats.csv conv3x3 $X >> $O/${TAG}_conv_exp.log
        done
      done
      cat $O/${TAG}_conv_exp.log ;;
    conv_tests) step conv_tests 900 $PYT -m gpu $R/tests/test_gpu_ops.py $R/tests/test_gpu_ln_side.py $R/tests/test_gpu_production_parity.py ;;
    conv_kern)
      # refine-conv kernel times, this build vs an override library (CONV_B)
      for L in "" "$CONV_B"; do
        for args in "1 6 bwd" "0 6 fwd act" "1 6 fwd"; do
          d=$O/${TAG}_convk_$(basename "${L:-cur}" .so)_${args// /_}
          MSU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/conv_one.py $args > /dev/null 2>&1 || exit 3
          python3 $R/tools/kstats.py $d/p_kernel_stats.csv conv3x3 "${L:+B}" >> $O/${TAG}_conv_kern.log
        done
      done
      cat $O/${TAG}_conv_kern.log ;;
    ab_wgrad) bash $R/tools/gpu_bench_ab.sh ${TAG}_wgrad "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_wgrad_256.so" \
                "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_wgrad_512.so" "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_wgrad_256.so" \
                "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_wgrad_512.so" || exit 3 ;;
    conv_env)
      # refine-conv kernel times under two environments (CONV_ENV_B, e.g. MSU_CONV_V5=0)
      for E in "NOENV=1" "$CONV_ENV_B"; do
        for args in "1 6 fwd act" "0 6 fwd act" "1 6 bwd"; do
          d=$O/${TAG}_conve_${E%%=*}_${args// /_}
          env $E timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/conv_one.py $args > /dev/null 2>&1 || exit 3
          python3 $R/tools/kstats.py $d/p_kernel_stats.csv conv3x3 "${E%%=*}" >> $O/${TAG}_conv_env.log
        done
      done
      cat $O/${TAG}_conv_env.log ;;
    ab_env) bash $R/tools/gpu_bench_ab.sh ${TAG}_env "" "$AB_ENV" "" "$AB_ENV" "" "$AB_ENV" || exit 3 ;;
    ab_env2) bash $R/tools/gpu_bench_ab.sh ${TAG}_env2 "" "$AB_ENV" "$AB_ENV2" "" "$AB_ENV" "$AB_ENV2" || exit 3 ;;
    mlp_s1_var)
      # stage-1 fused MLP variants (tools/build_exp.sh mlp_s1 1 2): kernel times, twice each
      for r in 1 2; do for L in "" $R/tools/exp/libmsunet_mlp_s1_1.so $R/tools/exp/libmsunet_mlp_s1_2.so; do
        echo "== ${L:-cur}" >> $O/${TAG}_mlp_s1_var.log
        MSU_LIB_OVERRIDE=$L timeout -k 10 200 python -u $R/tools/mlp_s1_one.py 20 2>&1 | grep fused >> $O/${TAG}_mlp_s1_var.log || exit 3
      done; done
      cat $O/${TAG}_mlp_s1_var.log ;;
    ln_exp)
      for X in ${LN_EXP:-0 1 2 8}; do
        L=""; [ $X != 0 ] && L=$R/tools/exp/libmsunet_layernorm_$X.so
        echo "== MSU_EXP=$X" >> $O/${TAG}_ln_exp.log
        for K in ln lnadd; do
          MSU_LIB_OVERRIDE=$L timeout -k 10 200 python -u $R/tools/kbench.py $K >> $O/${TAG}_ln_exp.log 2>&1 || exit 3
        done
      done
      cat $O/${TAG}_ln_exp.log ;;
    ln_kern)
      # LayerNorm kernel times at the step's shapes per ablation build (LN_EXP masks, 0 = this build)
      for X in ${LN_EXP:-0 16 32 64}; do
        L=""; [ $X != 0 ] && L=$R/tools/exp/libmsunet_layernorm_$X.so
        d=$O/${TAG}_lnk_$X
        MSU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/ln_one.py 5 > /dev/null 2>&1 || exit 3
        python3 $R/tools/kstats.py $d/p_kernel_stats.csv ln_ X$X >> $O/${TAG}_ln_kern.log
      done
      cat $O/${TAG}_ln_kern.log ;;
    ab_ln) bash $R/tools/gpu_bench_ab.sh ${TAG}_ln "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_layernorm_1.so" \
             "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_layernorm_2.so" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_layernorm_8.so" \
             "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_layernorm_1.so" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_layernorm_2.so" \
             "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_layernorm_8.so" || exit 3 ;;
    nt_store) step nt_store 400 bash $R/tools/nt_store_ab.sh ;;
    ab_lib) bash $R/tools/gpu_bench_ab.sh ${TAG}_lib "" "MSU_LIB_OVERRIDE=$AB_LIB" "" "MSU_LIB_OVERRIDE=$AB_LIB" "" "MSU_LIB_OVERRIDE=$AB_LIB" || exit 3 ;;
    tail_tests) step tail_tests 600 $PYT -m gpu $R/tests/test_gpu_tail_reduce.py $R/tests/test_gpu_ln_side.py \
                  $R/tests/test_gpu_tok_gemm.py $R/tests/test_gpu_linbwd.py ;;
    mlp_kern)
      # stage-0 no-grad MLP kernels: fused (MSU_MLP_INFER=1) vs the token-GEMM pair
      for X in 1 0; do
        d=$O/${TAG}_mlpk_$X
        MSU_MLP_INFER=$X timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/mlp_one.py 5 > /dev/null 2>&1 || exit 3
        python3 $R/tools/kstats.py $d/p_kernel_stats.csv gemm I$X >> $O/${TAG}_mlp_kern.log
        python3 $R/tools/kstats.py $d/p_kernel_stats.csv mlp I$X >> $O/${TAG}_mlp_kern.log
      done
      if [ -n "$AB_LIB" ]; then
        d=$O/${TAG}_mlpk_B
        MSU_LIB_OVERRIDE=$AB_LIB timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o p --output-format csv -- python3 $R/tools/mlp_one.py 5 > /dev/null 2>&1 || exit 3
        python3 $R/tools/kstats.py $d/p_kernel_stats.csv mlp B >> $O/${TAG}_mlp_kern.log
      fi
      cat $O/${TAG}_mlp_kern.log ;;
    mlp_pmc)
      # counters of the fused MLP (no-grad, 8 x 256^2 tokens): HBM bytes, VALU / MFMA / LDS activity
      d=$O/${TAG}_mlppmc
      for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA GRBM_GUI_ACTIVE"; do
        tagc=$(echo $c | cut -d' ' -f1)
        timeout -s KILL 90 rocprofv3 --pmc $c -d $d -o $tagc --output-format csv -- python3 $R/tools/mlp_one.py 3 > /dev/null 2>&1 || exit 3
      done
      for f in $d/*_counter_collection.csv; do python3 $R/tools/pmc_sum.py mlp_fused $f; done > $O/${TAG}_mlp_pmc.log
      cat $O/${TAG}_mlp_pmc.log ;;
    ab_aux) bash $R/tools/gpu_bench_ab.sh ${TAG}_aux "" "MSU_ATTN_AUX=0" "" "MSU_ATTN_AUX=0" "" "MSU_ATTN_AUX=0" || exit 3 ;;
    ab_mlp_ln) bash $R/tools/gpu_bench_ab.sh ${TAG}_mlpln "" "MSU_MLP_LN=0" "" "MSU_MLP_LN=0" "" "MSU_MLP_LN=0" || exit 3 ;;
    ab_mlp_train) bash $R/tools/gpu_bench_ab.sh ${TAG}_mlptrain "" "MSU_MLP_TRAIN=0" "" "MSU_MLP_TRAIN=0" "" "MSU_MLP_TRAIN=0" || exit 3 ;;
    ab_mlp) bash $R/tools/gpu_bench_ab.sh ${TAG}_mlp "" "MSU_MLP_INFER=0" "" "MSU_MLP_INFER=0" "" "MSU_MLP_INFER=0" || exit 3 ;;
    ab_tail) bash $R/tools/gpu_bench_ab.sh ${TAG}_tail "" "MSU_TAIL=0" "" "MSU_TAIL=0" "" "MSU_TAIL=0" || exit 3 ;;
    ab_fused) bash $R/tools/gpu_bench_ab.sh ${TAG}_fused "" "MSU_ATTN_QKV=0" "" "MSU_ATTN_QKV=0" "" "MSU_ATTN_QKV=0" || exit 3 ;;
    determ) step determ 600 python -u $R/tools/determinism_matrix.py 24 default ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done

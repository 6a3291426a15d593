# One GPU call, named steps run in order, each under its own time limit; the call stops at the
# first step that faults, aborts or times out (exit status > 1).  Logs: gpurun_out/TAG_<step>.log
#   bash tools/gpu_call.sh TAG step [step ...]
# steps: tests_new (the round's new GPU tests), tests (whole -m gpu suite), bench,
#        wgrad_ab (wgrad timing, XCD-grouped vs linear grid), wgrad_pmc (HBM counters, both),
#        prof (eager step under rocprofv3 --kernel-trace --stats)
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
    fused_tests) step fused_tests 300 $PYT -m gpu $R/tests/test_gpu_attn_qkv.py ;;
    tests_new) step tests_new 600 $PYT -m gpu $R/tests/test_gpu_production_parity.py $R/tests/test_gpu_bench_dp.py \
                 $R/tests/test_gpu_linbwd.py "$R/tests/test_gpu_tok_gemm.py::test_linear_cat_direct_grad_accumulates" \
                 "$R/tests/test_gpu_graph.py::test_eager_side_stream_step_is_deterministic" ;;
    tests) step tests 900 python -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    bench) step bench 480 python -u $R/bench.py
           grep '^{' $O/${TAG}_bench.log > $O/${TAG}_bench.json ;;
    wgrad_ab)
      for x in 1 0 1 0; do
        for shp in "32768 1152 384" "32768 384 1536" "131072 576 192" "8192 2304 768" "131072 192 768"; do
          MSU_WGRAD_XCD=$x timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 50 >> $O/${TAG}_wgrad_ab.log 2>&1 || exit 3
          echo "xcd=$x" >> $O/${TAG}_wgrad_ab.log
        done
      done
      tail -20 $O/${TAG}_wgrad_ab.log ;;
    wgrad_pmc)
      for x in 1 0; do
        for c in FETCH_SIZE WRITE_SIZE; do
          MSU_WGRAD_XCD=$x timeout -s KILL 90 rocprofv3 --pmc $c -d $O/${TAG}_wpmc_${x}_$c -o p --output-format csv -- \
            python3 $R/tools/wgrad_one.py 32768 1152 384 10 > $O/${TAG}_wpmc_${x}_$c.log 2>&1 || exit 3
        done
      done ;;
    conv_ab)
      for v in "" 16 "" 16; do
        echo "MSU_CONV_MFMA=$v" >> $O/${TAG}_conv_ab.log
        MSU_CONV_MFMA=$v timeout -k 10 180 python -u $R/tools/kbench.py conv >> $O/${TAG}_conv_ab.log 2>&1 || exit 3
      done
      tail -12 $O/${TAG}_conv_ab.log ;;
    conv16_tests) MSU_CONV_MFMA=16 step conv16_tests 400 $PYT -m gpu $R/tests/test_gpu_production_parity.py -k refine \
                    $R/tests/test_gpu_ops.py -k "refine_conv_act" ;;
    wgrad_split)
      for sp in "" "1,1" "2,1" "4,1"; do
        echo "MSU_WGRAD_SPLIT=$sp" >> $O/${TAG}_wgrad_split.log
        MSU_WGRAD_SPLIT=$sp timeout -k 10 60 python -u $R/tools/wgrad_one.py 32768 1152 384 50 >> $O/${TAG}_wgrad_split.log 2>&1 || exit 3
        for c in FETCH_SIZE WRITE_SIZE; do
          MSU_WGRAD_SPLIT=$sp timeout -s KILL 90 rocprofv3 --pmc $c -d $O/${TAG}_wsp_${sp/,/_}_$c -o p --output-format csv -- \
            python3 $R/tools/wgrad_one.py 32768 1152 384 10 > /dev/null 2>&1 || exit 3
        done
      done
      tail -8 $O/${TAG}_wgrad_split.log ;;
    nt_ab)
      for r in 1 2; do
        for bn in 128 192; do
          for shp in "32768 384 384" "32768 384 1152" "32768 384 1536" "32768 1152 384" "131072 192 768" "131072 576 192" "32000 384 192"; do
            echo -n "bn=$bn " >> $O/${TAG}_nt_ab.log
            MSU_NT_BN=$bn timeout -k 10 60 python -u $R/tools/nt_one.py $shp 50 >> $O/${TAG}_nt_ab.log 2>&1 || exit 3
          done
        done
      done
      tail -14 $O/${TAG}_nt_ab.log ;;
    attn_pmc) step attn_pmc 400 bash $R/tools/pmc_attn.sh $TAG 256 3 3 0.05 ;;
    fused_ab)
      for r in 1 2 3; do
        for v in 1 0; do
          echo "MSU_ATTN_QKV=$v" >> $O/${TAG}_fused_ab.log
          MSU_ATTN_QKV=$v timeout -k 10 240 python3 -u $R/bench.py --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --no-input-pipeline 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> $O/${TAG}_fused_ab.log || exit 3
        done
      done
      cat $O/${TAG}_fused_ab.log ;;
    wgrad_nst)
      for shp in "32768 1152 384" "32768 384 384" "32768 1536 384" "32768 384 1536" "131072 576 192" "131072 192 192" \
                 "131072 768 192" "131072 192 768" "8192 2304 768" "8192 3072 768" "8192 768 3072" "524288 288 96"; do
        for nst in 3 4 5 6; do
          echo -n "NST=$nst " >> $O/${TAG}_wgrad_nst.log
          MSU_WGRAD_NST=$nst timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 30 2>&1 | grep wgrad >> $O/${TAG}_wgrad_nst.log || exit 3
        done
      done
      cat $O/${TAG}_wgrad_nst.log ;;
    wgrad_diag)
      for shp in "32768 1152 384" "8192 2304 768" "131072 576 192"; do
        for lib in "" $R/tools/exp/libmsunet_gemm_wgrad_1.so $R/tools/exp/libmsunet_gemm_wgrad_2.so; do
          echo -n "lib=${lib##*/} " >> $O/${TAG}_wgrad_diag.log
          MSU_LIB_OVERRIDE=$lib timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 30 2>&1 | grep wgrad >> $O/${TAG}_wgrad_diag.log || exit 3
        done
      done
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
        -d $O/${TAG}_wgpmc1 -o p --output-format csv -- python3 $R/tools/wgrad_one.py 32768 1152 384 10 > /dev/null 2>&1 || exit 3
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
        -d $O/${TAG}_wgpmc2 -o p --output-format csv -- python3 $R/tools/wgrad_one.py 32768 1152 384 10 > /dev/null 2>&1 || exit 3
      cat $O/${TAG}_wgrad_diag.log ;;
    vform_tests) MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_vform.so step vform_tests 900 python -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    vform_kern)
      for lib in "" $R/tools/exp/libmsunet_vform.so "" $R/tools/exp/libmsunet_vform.so; do
        echo "lib=${lib##*/}" >> $O/${TAG}_vform_kern.log
        for shp in "32768 1152 384" "8192 2304 768" "131072 576 192" "524288 288 96"; do
          MSU_LIB_OVERRIDE=$lib timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 30 2>&1 | grep wgrad >> $O/${TAG}_vform_kern.log || exit 3
        done
        for shp in "32768 1152 384" "131072 192 576" "8192 768 3072"; do
          MSU_LIB_OVERRIDE=$lib timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_vform_kern.log || exit 3
        done
      done
      cat $O/${TAG}_vform_kern.log ;;
    vform_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_vform "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_vform.so" "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_vform.so" "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_vform.so" || exit 3 ;;
    kern)
      for shp in "32768 1152 384" "8192 2304 768" "131072 576 192" "524288 288 96"; do
        timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 30 2>&1 | grep wgrad >> $O/${TAG}_kern.log || exit 3
      done
      for shp in "32768 1152 384" "131072 192 576" "8192 768 3072"; do
        timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_kern.log || exit 3
      done
      cat $O/${TAG}_kern.log ;;
    attn_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_attn "" "MSU_ATTN_BWD_HPW=1" "" "MSU_ATTN_BWD_HPW=1" "" "MSU_ATTN_BWD_HPW=1" || exit 3 ;;
    skipw_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_skipw "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_wgrad_256.so" "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_wgrad_256.so" || exit 3 ;;
    nt_tile)
      for shp in "32768 1152 384" "32768 384 384" "32768 1536 384" "32768 384 1536" "131072 576 192" "131072 192 768" "8192 2304 768" "8192 768 3072"; do
        for t in "256 192" "128 192" "192 192" "256 128" "128 128"; do
          set -- $t
          echo -n "tile=$1x$2 " >> $O/${TAG}_nt_tile.log
          MSU_NT_TILE=$1 MSU_NT_BN=$2 timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_nt_tile.log || exit 3
        done
      done
      cat $O/${TAG}_nt_tile.log ;;
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
    ntbk_tests) MSU_NT_BK=32 step ntbk_tests 400 $PYT -m gpu $R/tests/test_gpu_nt_gemm.py $R/tests/test_gpu_tok_gemm.py $R/tests/test_gpu_baseline_shapes.py ;;
    ntbk_kern)
      for shp in "32768 1152 384" "32768 384 384" "32768 1536 384" "32768 384 1536" "131072 576 192" "131072 192 768" "8192 2304 768" "8192 768 3072"; do
        for bk in 64 32 64 32; do
          echo -n "bk=$bk " >> $O/${TAG}_ntbk.log
          MSU_NT_BK=$bk timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_ntbk.log || exit 3
        done
      done
      cat $O/${TAG}_ntbk.log ;;
    ntbk_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_ntbk "" "MSU_NT_BK=32" "" "MSU_NT_BK=32" "" "MSU_NT_BK=32" || exit 3 ;;
    nt192_tests) MSU_NT_TILE=192 MSU_NT_BN=192 step nt192_tests 400 $PYT -m gpu $R/tests/test_gpu_nt_gemm.py -k "not underfilled and not chosen" ;;
    dma_probe) step dma_probe 120 python -u $R/tools/dma_probe.py ;;
    ntsb_ab)
      for lib in "" $R/tools/exp/libmsunet_gemm_nt_0.so "" $R/tools/exp/libmsunet_gemm_nt_0.so; do
        echo "lib=${lib##*/}" >> $O/${TAG}_ntsb.log
        for shp in "32768 1152 384" "32768 384 384" "32768 384 1536" "131072 576 192" "131072 192 768" "8192 2304 768" "8192 768 3072"; do
          MSU_LIB_OVERRIDE=$lib timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_ntsb.log || exit 3
        done
      done
      cat $O/${TAG}_ntsb.log
      bash $R/tools/gpu_bench_ab.sh ${TAG}_ntsb "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_nt_0.so" "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_nt_0.so" || exit 3 ;;
    glds_ab)
      for lib in "" $R/tools/exp/libmsunet_gldsb.so "" $R/tools/exp/libmsunet_gldsb.so; do
        echo "lib=${lib##*/}" >> $O/${TAG}_glds.log
        for shp in "32768 1152 384" "32768 384 1536" "131072 192 768" "8192 768 3072"; do
          MSU_LIB_OVERRIDE=$lib timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" >> $O/${TAG}_glds.log || exit 3
        done
        MSU_LIB_OVERRIDE=$lib timeout -k 10 180 python -u $R/tools/kbench.py conv >> $O/${TAG}_glds.log 2>&1 || exit 3
      done
      cat $O/${TAG}_glds.log
      bash $R/tools/gpu_bench_ab.sh ${TAG}_glds "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gldsb.so" "" "MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gldsb.so" || exit 3 ;;
    w8_ab)
      for v in 1 0 1 0; do
        echo "MSU_WGRAD_W8=$v" >> $O/${TAG}_w8.log  # (default 0)
        for shp in "32768 1152 384" "8192 2304 768" "131072 576 192" "32768 384 1536" "8192 768 3072" "131072 192 768"; do
          MSU_WGRAD_W8=$v timeout -k 10 60 python -u $R/tools/wgrad_one.py $shp 30 2>&1 | grep wgrad >> $O/${TAG}_w8.log || exit 3
        done
      done
      cat $O/${TAG}_w8.log
      bash $R/tools/gpu_bench_ab.sh ${TAG}_w8 "MSU_WGRAD_W8=1" "" "MSU_WGRAD_W8=1" "" || exit 3 ;;
    conv_pmc)
      timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/${TAG}_pmcconv -o conv_fetch --output-format csv -- python3 $R/tools/conv_one.py 0 3 fwd act > /dev/null 2>&1 || exit 3
      timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/${TAG}_pmcconv -o conv_write --output-format csv -- python3 $R/tools/conv_one.py 0 3 fwd act > /dev/null 2>&1 || exit 3
      python3 $R/tools/pmc_json.py conv3x3_v3_kernel $O/${TAG}_pmcconv/conv_fetch_counter_collection.csv \
        $O/${TAG}_pmcconv/conv_write_counter_collection.csv $O/${TAG}_conv3x3_fwd_pmc.json && cat $O/${TAG}_conv3x3_fwd_pmc.json ;;
    cat_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_cat "" "MSU_CAT_SIDE=0" "" "MSU_CAT_SIDE=0" "" "MSU_CAT_SIDE=0" || exit 3 ;;
    determ) step determ 600 python -u $R/tools/determinism_matrix.py 24 default ;;
    conv_side_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_convside "" "MSU_CONV_SIDE=0" "" "MSU_CONV_SIDE=0" "" "MSU_CONV_SIDE=0" || exit 3 ;;
    defer_tests) step defer_tests 300 $PYT -m gpu $R/tests/test_gpu_ln_side.py $R/tests/test_gpu_trainer.py $R/tests/test_gpu_rccl.py $R/tests/test_gpu_graph.py ;;
    defer_tests1) MSU_CONV_DEFER=1 step defer_tests1 300 $PYT -m gpu $R/tests/test_gpu_trainer.py $R/tests/test_gpu_rccl.py $R/tests/test_gpu_graph.py $R/tests/test_gpu_bench_dp.py ;;
    defer_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_defer "MSU_CONV_DEFER=1" "" "MSU_CONV_DEFER=1" "" "MSU_CONV_DEFER=1" "" || exit 3 ;;
    lnpf_iso) MSU_LN_FWD_PF=0 MSU_LN_BWD_PF=0 step lnpf_save 120 python -u $R/tools/ln_pf_check.py save $O/${TAG}_ln0.pt && \
              MSU_LN_FWD_PF=0 MSU_LN_BWD_PF=0 step lnpf_same 120 python -u $R/tools/ln_pf_check.py compare $O/${TAG}_ln0.pt && \
              MSU_LN_BWD_PF=0 step lnpf_fwdonly 120 python -u $R/tools/ln_pf_check.py compare $O/${TAG}_ln0.pt && \
              MSU_LN_FWD_PF=0 step lnpf_bwdonly 120 python -u $R/tools/ln_pf_check.py compare $O/${TAG}_ln0.pt && \
              step lnpf_both 120 python -u $R/tools/ln_pf_check.py compare $O/${TAG}_ln0.pt ;;
    headpf) MSU_HEAD_BWD_PF=0 step headpf_save 120 python -u $R/tools/ln_pf_check.py save $O/${TAG}_h0.pt && \
            step headpf_check 120 python -u $R/tools/ln_pf_check.py compare $O/${TAG}_h0.pt && \
            step headpf_tests 300 $PYT -m gpu $R/tests/test_gpu_ops.py -k "head or norm" ;;
    headpf_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_headpf "" "MSU_HEAD_BWD_PF=0" "" "MSU_HEAD_BWD_PF=0" "" "MSU_HEAD_BWD_PF=0" || exit 3 ;;
    convblk_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_convblk "" "MSU_CONV_WGRAD_BLOCKS=192" "MSU_CONV_WGRAD_BLOCKS=128" "" "MSU_CONV_WGRAD_BLOCKS=192" "MSU_CONV_WGRAD_BLOCKS=128" || exit 3 ;;
    convblk_tests) MSU_CONV_WGRAD_BLOCKS=128 step convblk_tests 300 $PYT -m gpu $R/tests/test_gpu_ln_side.py $R/tests/test_gpu_ops.py -k "refine or conv" ;;
    lnpf_check) MSU_LN_FWD_PF=0 MSU_LN_BWD_PF=0 step lnpf_save 120 python -u $R/tools/ln_pf_check.py save $O/${TAG}_ln0.pt && \
                step lnpf_check 120 python -u $R/tools/ln_pf_check.py compare $O/${TAG}_ln0.pt && \
                step lnpf_tests 300 $PYT -m gpu $R/tests/test_gpu_ops.py -k "norm" $R/tests/test_gpu_ln_side.py ;;
    lnpf_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_lnpf "" "MSU_LN_BWD_PF=0" "" "MSU_LN_BWD_PF=0" "" "MSU_LN_BWD_PF=0" || exit 3 ;;
    lnfpf_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_lnfpf "" "MSU_LN_FWD_PF=0" "" "MSU_LN_FWD_PF=0" "" "MSU_LN_FWD_PF=0" || exit 3 ;;
    lndeep_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_lndeep "" "MSU_LN_PARTS_DEEP=512" "MSU_LN_PARTS_DEEP=256" "" "MSU_LN_PARTS_DEEP=512" "MSU_LN_PARTS_DEEP=256" || exit 3 ;;
    lnparts_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_lnparts "" "MSU_LN_PARTS_MAX=512" "MSU_LN_PARTS_MAX=256" "" "MSU_LN_PARTS_MAX=512" "MSU_LN_PARTS_MAX=256" || exit 3 ;;
    ln_ab) bash $R/tools/gpu_bench_ab.sh ${TAG}_ln "MSU_LN_SIDE=1" "" "MSU_LN_SIDE=1" "" "MSU_LN_SIDE=1" "" || exit 3 ;;
    fused3_ab)
      for r in 1 2; do
        for v in hs 1 0; do
          echo "MSU_ATTN_QKV=$v" >> $O/${TAG}_fused3_ab.log
          MSU_ATTN_QKV=$v timeout -k 10 240 python3 -u $R/bench.py --steps 15 --warmup 5 --no-cpu-baseline --no-input-pipeline 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('roofline_attention', {}).get('fused_unit')))" >> $O/${TAG}_fused3_ab.log || exit 3
        done
      done
      cat $O/${TAG}_fused3_ab.log ;;
    nt_tests) step nt_tests 400 $PYT -m gpu $R/tests/test_gpu_nt_gemm.py $R/tests/test_routing.py ;;
    nt_pmc)
      timeout -k 10 60 python -u $R/tools/nt_one.py 32768 1152 384 50 > $O/${TAG}_nt.log 2>&1 || exit 3
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
        -d $O/${TAG}_ntpmc1 -o p --output-format csv -- python3 $R/tools/nt_one.py 32768 1152 384 10 >> $O/${TAG}_nt.log 2>&1 || exit 3
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
        -d $O/${TAG}_ntpmc2 -o p --output-format csv -- python3 $R/tools/nt_one.py 32768 1152 384 10 >> $O/${TAG}_nt.log 2>&1 || exit 3
      cat $O/${TAG}_nt.log | grep "nt M" ;;
    # MSU_GRAPH=0: the profiler's per-launch host cost makes the bench's auto policy pick the
    # single-stream graph replay; the profile must show the eager step the bench line measures
    prof) MSU_GRAPH=0 step prof 420 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o p --output-format csv -- \
            python3 $R/bench.py --steps 8 --warmup 4 --no-roofline --no-cpu-baseline --no-input-pipeline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done

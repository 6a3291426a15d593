# Memory-pipeline stall counters over token-GEMM shapes: bash tools/pmc_tok2.sh "M N K epi" ...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for spec in "$@"; do
  set -- $spec
  O=$R/gpurun_out/pmc2_$1_$2_$3_$4
  mkdir -p $O
  i=0
  for ctrs in "GRBM_GUI_ACTIVE TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCC_EA0_WRREQ_STALL TCC_TAG_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL" \
              "TA_DATA_STALLED_BY_TC_CYCLES TA_FLAT_WRITE_WAVEFRONTS TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT" \
              "TCP_TCC_WRITE_REQ_LATENCY TCP_TCC_READ_REQ_LATENCY TCP_TCC_WRITE_REQ TCP_TCC_READ_REQ TCC_BUSY TCC_HIT TCC_MISS"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $ctrs -d $O -o p$i --output-format csv -- python3 $R/tools/tok_one.py $1 $2 $3 $4 3 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  done
  echo "== $spec"
  for f in $O/p*_counter_collection.csv; do python3 $R/tools/pmc_sum.py tokgemm $f; done
done

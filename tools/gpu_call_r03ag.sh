# r03ag: round-3 final evidence (tests, bench, step profile, conv / wgrad counters, graph probe) +
# HBM counters of the one-pass Linear backward at the qkv shape
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
bash $R/tools/gpu_round3.sh r03ag || exit $?
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 90 rocprofv3 --pmc $c -d $O/pmc_r03ag -o linbwd_$c --output-format csv -- \
      python3 $R/tools/linbwd_bench.py 96 288 > $O/r03ag_pmc_linbwd_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 $R/tools/pmc_json.py linbwd_kernel $O/pmc_r03ag/linbwd_FETCH_SIZE_counter_collection.csv \
    $O/pmc_r03ag/linbwd_WRITE_SIZE_counter_collection.csv $O/r03ag_linbwd_96_288_pmc.json
cat $O/r03ag_linbwd_96_288_pmc.json

# Round-3 evidence in one GPU call: parity tests, the bench line, the kernel-trace profile of
# the eager step, HBM counters (separate FETCH_SIZE / WRITE_SIZE passes) of the roofline conv
# and of the Linear weight-gradient kernel at a stage-0 and a stage-2 shape.
#   bash tools/gpu_round3.sh TAG
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() {  # name seconds cmd...  (stop the call on a fault / abort / time-out)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/${TAG}_$name.log 2>&1
  local rc=$?
  tail -3 $O/${TAG}_$name.log
  echo "== $name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step gpu_tests 500 python -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench 420 python -u $R/bench.py
grep '^{' $O/${TAG}_bench.log > $O/${TAG}_bench.json
step prof 300 env MSU_GRAPH=0 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --steps 4 --warmup 4 --no-cpu-baseline --no-roofline --no-input-pipeline
python3 $R/tools/stream_summary.py $O/prof_$TAG/run_kernel_trace.csv > $O/${TAG}_streams.txt
python3 $R/tools/profsum.py $O/prof_$TAG/run_kernel_stats.csv 8 40 > $O/${TAG}_summary.txt
step pmc_conv_f 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$TAG -o conv_fetch --output-format csv -- \
    python3 $R/tools/conv_one.py 0 3 fwd act
step pmc_conv_w 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$TAG -o conv_write --output-format csv -- \
    python3 $R/tools/conv_one.py 0 3 fwd act
python3 $R/tools/pmc_json.py conv3x3_v3_kernel $O/pmc_$TAG/conv_fetch_counter_collection.csv \
    $O/pmc_$TAG/conv_write_counter_collection.csv $O/${TAG}_conv3x3_fwd_pmc.json
for shape in "524288 288 96" "32768 1152 384"; do
  set -- $shape
  n=wgrad_$1_$2_$3
  step pmc_${n}_f 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$TAG -o ${n}_fetch --output-format csv -- \
      python3 $R/tools/wgrad_one.py $1 $2 $3 5
  step pmc_${n}_w 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$TAG -o ${n}_write --output-format csv -- \
      python3 $R/tools/wgrad_one.py $1 $2 $3 5
  step pmc_${n}_sq 90 rocprofv3 --kernel-trace --stats -d $O/pmc_$TAG -o ${n}_trace --output-format csv -- \
      python3 $R/tools/wgrad_one.py $1 $2 $3 5
  python3 $R/tools/pmc_json.py wgrad_wave_kernel $O/pmc_$TAG/${n}_fetch_counter_collection.csv \
      $O/pmc_$TAG/${n}_write_counter_collection.csv $O/${TAG}_${n}_pmc.json
done
step probe 300 env MSU_GRAPH_SIDE=1 python -u $R/tools/graph_side_probe.py 5
echo done

# One GPU call: parity tests, bench line, kernel-trace profile, HBM counter passes on the
# roofline kernel.  Usage (from the repo root, on the GPU box):  bash tools/gpu_round.sh TAG
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "== bench"
timeout -k 10 300 python -u $R/bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -30 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
echo "== rocprof kernel trace"
# eager (the bench's own choice at 1024^2; under the profiler the auto policy would capture)
MSU_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-input-pipeline > $O/prof_$TAG.log 2>&1 || { tail -30 $O/prof_$TAG.log; exit 1; }
python3 $R/tools/stream_summary.py $O/prof_$TAG/run_kernel_trace.csv > $O/streams_$TAG.txt
echo "== HBM counters (conv fwd)"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$TAG -o fetch --output-format csv -- \
    python3 $R/tools/conv_one.py 0 3 fwd act > $O/pmc_$TAG.log 2>&1 || { tail -20 $O/pmc_$TAG.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$TAG -o write --output-format csv -- \
    python3 $R/tools/conv_one.py 0 3 fwd act >> $O/pmc_$TAG.log 2>&1 || { tail -20 $O/pmc_$TAG.log; exit 1; }
python3 $R/tools/pmc_json.py conv3x3_v2_kernel $O/pmc_$TAG/fetch_counter_collection.csv \
    $O/pmc_$TAG/write_counter_collection.csv $O/conv3x3_fwd_pmc_$TAG.json
python3 $R/tools/profsum.py $O/prof_$TAG/run_kernel_stats.csv 6 40
echo done

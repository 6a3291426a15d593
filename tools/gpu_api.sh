set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/prof_api -o run --output-format csv -- \
    python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-input-pipeline > $O/prof_api.log 2>&1 || { tail -30 $O/prof_api.log; exit 1; }
ls $O/prof_api
python3 $R/tools/api_summary.py $O/prof_api/run_hip_api_trace.csv $O/prof_api/run_kernel_trace.csv > $O/api.txt
rm -f $O/prof_api/run_hip_api_trace.csv

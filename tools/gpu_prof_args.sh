# Kernel + HIP API trace of bench with extra args:  bash tools/gpu_prof_args.sh TAG [bench args]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-input-pipeline "$@" > $O/prof_$TAG.log 2>&1 || { tail -30 $O/prof_$TAG.log; exit 1; }
python3 $R/tools/api_summary.py $O/prof_$TAG/run_hip_api_trace.csv $O/prof_$TAG/run_kernel_trace.csv > $O/${TAG}_api.txt
python3 $R/tools/gap_summary.py $O/prof_$TAG/run_kernel_trace.csv 25 > $O/${TAG}_gaps.txt
python3 $R/tools/profsum.py $O/prof_$TAG/run_kernel_stats.csv 4 30 > $O/${TAG}_summary.txt
rm -f $O/prof_$TAG/run_hip_api_trace.csv

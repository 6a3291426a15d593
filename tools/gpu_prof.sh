# Kernel-trace profile of the bench step: bash tools/gpu_prof.sh TAG
set -e
TAG=${1:-x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-input-pipeline > $O/prof_$TAG.log 2>&1 || { tail -30 $O/prof_$TAG.log; exit 1; }
python3 $R/tools/profsum.py $O/prof_$TAG/run_kernel_stats.csv 6 45

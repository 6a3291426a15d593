# Kernel-trace profile of the bench step with the NT GEMM routed in (per-stream view), to compare
# its in-step kernel times with tools/kbench.py nt:  bash tools/nt_step_prof.sh TAG
set -e
TAG=${1:-nt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MSU_GRAPH=0 MSU_GEMM_ROUTE=nt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-input-pipeline > $O/prof_$TAG.log 2>&1 || { tail -30 $O/prof_$TAG.log; exit 1; }
python3 $R/tools/stream_summary.py $O/prof_$TAG/run_kernel_trace.csv > $O/streams_$TAG.txt
head -60 $O/streams_$TAG.txt

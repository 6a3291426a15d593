# Same-box A/B of an environment switch on the bench (eager step), interleaved:
#   bash tools/gpu_ab.sh TAG "ENV_A" "ENV_B" [pairs] [steps]
# e.g. bash tools/gpu_ab.sh st "MSU_SHADOW_T=1" "MSU_SHADOW_T=0" 2
TAG=$1; A=$2; B=$3; PAIRS=${4:-2}; STEPS=${5:-15}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python -u $R/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-roofline --no-input-pipeline"
for i in $(seq 1 $PAIRS); do
  for arm in a b; do
    if [ $arm = a ]; then E=$A; else E=$B; fi
    timeout -k 10 240 env MSU_GRAPH=0 $E $CMD > $O/${TAG}_ab_${arm}$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -20 $O/${TAG}_ab_${arm}$i.log; exit $rc; fi
    echo "$arm$i [$E] $(grep -o '"value": [0-9.]*' $O/${TAG}_ab_${arm}$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/${TAG}_ab_${arm}$i.log)"
  done
done

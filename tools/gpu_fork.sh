# Forked-stream HIP graph: bisect its nondeterminism by side-stream use, then what the forked
# replay would buy at the bench shape (eager vs single-stream replay vs forked replay).
#   bash tools/gpu_fork.sh TAG
TAG=${1:-fork}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() {  # name seconds cmd...  (stop the call on a fault / abort / time-out)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/${TAG}_$name.log 2>&1
  local rc=$?
  tail -8 $O/${TAG}_$name.log
  echo "== $name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step bisect 420 python -u $R/tools/graph_fork_bisect.py 5
B="python -u $R/bench.py --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --no-input-pipeline"
step eager 200 env MSU_GRAPH=0 $B
step replay1 200 env MSU_GRAPH=1 $B
step replay_fork 200 env MSU_GRAPH=1 MSU_GRAPH_SIDE=1 $B
step eager_b 200 env MSU_GRAPH=0 $B
step replay_fork_b 200 env MSU_GRAPH=1 MSU_GRAPH_SIDE=1 $B
for n in eager replay1 replay_fork eager_b replay_fork_b; do
  echo "$n $(grep -o '"value": [0-9.]*' $O/${TAG}_$n.log) $(grep -o '"host_ms_per_step": [0-9.]*' $O/${TAG}_$n.log)"
done
echo done

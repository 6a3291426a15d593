# Eager vs HIP-graph replay of the bench step for one config, interleaved:
#   bash tools/graph_cfg_ab.sh N "bench args"
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; ARGS=$2
cd /tmp && export TMPDIR=/tmp
for i in $(seq $N); do
  for G in 0 1; do
    printf '[MSU_GRAPH=%s] ' $G
    MSU_GRAPH=$G timeout -k 10 300 python3 -u $R/bench.py --steps 10 --warmup 6 --no-cpu-baseline --no-roofline --no-input-pipeline $ARGS 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_ms_per_step'], d['config']['step_execution'])" || exit 1
  done
done

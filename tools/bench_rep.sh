# Bench N times in one GPU call (box-noise check): bash tools/bench_rep.sh N [extra bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; shift
cd /tmp && export TMPDIR=/tmp
for i in $(seq $N); do
  timeout -k 10 300 python3 -u $R/bench.py --no-cpu-baseline --no-roofline --no-input-pipeline "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
done

# Same-box A/B of the whole bench step under two environments, interleaved: bash tools/route_ab.sh N "ENV_A" "ENV_B"
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=$1; A=$2; B=$3
cd /tmp && export TMPDIR=/tmp
for i in $(seq $N); do
  for E in "$A" "$B"; do
    printf '%-28s ' "[${E:-default}]"
    env $E timeout -k 10 300 python3 -u $R/bench.py --steps 15 --warmup 4 --no-cpu-baseline --no-roofline --no-input-pipeline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done

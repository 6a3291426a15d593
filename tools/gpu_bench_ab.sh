# Same-box bench A/B over environment settings / bench flags, interleaved:
#   bash tools/gpu_bench_ab.sh TAG "ENV=.. [--flag]" "ENV=.." ...   (arm = env assignments then bench flags)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
TAG=$1; shift
for arm in "$@"; do
  envs=""; flags=""
  for w in $arm; do case $w in --*) flags="$flags $w";; *) envs="$envs $w";; esac; done
  echo "== $arm"
  env $envs timeout -k 10 240 python3 -u $R/bench.py --steps 15 --warmup 5 --no-cpu-baseline --no-roofline --no-input-pipeline $flags 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_ms_per_step'))" || exit 1
done > $O/${TAG}_bench_ab.log
cat $O/${TAG}_bench_ab.log

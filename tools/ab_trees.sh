# Same-box bench A/B of source trees (this tree and older ones checked out with their own built
# libraries, e.g. git worktrees of earlier commits), interleaved round by round:
#   bash tools/ab_trees.sh TAG ROUNDS DIR [DIR ...]      (DIR relative to this tree; "." = this tree)
# env: STEPS (default 15) timed steps per run.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
for i in $(seq $N); do
  for T in "$@"; do
    echo "== $T"
    timeout -k 10 240 python3 -u $R/$T/bench.py --steps ${STEPS:-15} --warmup 5 --no-cpu-baseline --no-roofline \
      --no-input-pipeline 2>&1 | grep '^{' \
      | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_ms_per_step'))" || exit 1
  done
done > $O/${TAG}_trees_ab.log
cat $O/${TAG}_trees_ab.log

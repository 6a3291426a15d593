# Quick GPU check of HEAD: the -m gpu suite and one bench line.
#   bash tools/gpu_check.sh TAG
TAG=${1:-chk}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() {  # name seconds cmd...  (stop the call on a fault / abort / time-out)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/${TAG}_$name.log 2>&1
  local rc=$?
  tail -3 $O/${TAG}_$name.log
  echo "== $name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step gpu_tests 600 python -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench 420 python -u $R/bench.py
grep '^{' $O/${TAG}_bench.log > $O/${TAG}_bench.json
if [ -n "$EXP" ]; then  # optional ablation timing: EXP="mode src mask..."
  step exp 400 bash $R/tools/exp_run.sh $EXP
fi
echo done

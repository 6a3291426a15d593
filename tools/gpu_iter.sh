# Iteration GPU call: selected tests, kbench modes, optional bench.  bash tools/gpu_iter.sh "<pytest -k expr or file>" "<kbench modes>" [bench]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$1" ]; then
  echo "== pytest $1"
  timeout -k 10 400 python -u -m pytest $R/$1 -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
     > $O/iter_pytest.log 2>&1 || { tail -40 $O/iter_pytest.log; exit 1; }
  tail -3 $O/iter_pytest.log
fi
for m in $2; do
  echo "== kbench $m"
  timeout -k 10 300 python -u $R/tools/kbench.py $m 2>&1 | tee $O/kbench_$m.log | grep -v Warning
done
if [ "$3" = "bench" ]; then
  echo "== bench"
  timeout -k 10 300 python -u $R/bench.py --no-cpu-baseline --no-input-pipeline > $O/iter_bench.json 2> $O/iter_bench.err || { tail -30 $O/iter_bench.err; exit 1; }
  cat $O/iter_bench.json
fi

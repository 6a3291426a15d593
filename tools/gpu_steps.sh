# Run GPU steps in order, each under its own time limit, stopping at the first step that
# faults / aborts / times out (exit >= 124 or a signal); a plain test failure (rc 1) goes on.
#   bash tools/gpu_steps.sh "NAME|SECONDS|COMMAND" ...      (outputs in gpurun_out/NAME.log)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export R O
status=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 $secs bash -c "$cmd" > $O/$name.log 2>&1
  rc=$?
  tail -4 $O/$name.log
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then status=$rc; fi
  if [ $rc -gt 2 ] && [ $rc -ne 5 ]; then
    echo "stopping: $name ended with $rc"
    exit $rc
  fi
done
exit $status

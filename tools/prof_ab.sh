# Eager kernel-trace profiles of the bench step under two environments; per-kernel per-step diff.
#   bash tools/prof_ab.sh "ENV_A" "ENV_B" [filter]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_ab
mkdir -p $O
i=0
for E in "$1" "$2"; do
  i=$((i+1))
  env MSU_GRAPH=0 $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$i -o run --output-format csv -- \
      python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-input-pipeline > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/p$i.log
done
python3 $R/tools/prof_diff.py $O/p1/run_kernel_stats.csv $O/p2/run_kernel_stats.csv 6 "${3:-}"

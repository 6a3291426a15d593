# Bench lines of the other single-GPU configs (BASELINE configs 2 and 5, Swin-B): bash tools/configs_bench.sh
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for args in "--img 512 --backbone swin_t" "--img 1024 --backbone swin_s" "--img 1024 --backbone swin_b"; do
  echo "== $args"
  timeout -k 10 300 python3 -u $R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-roofline --no-input-pipeline $args 2>&1 | grep '^{' >> $O/${TAG:-r06ax}_configs_bench.jsonl || exit 1
  tail -1 $O/${TAG:-r06ax}_configs_bench.jsonl | cut -c1-200
done

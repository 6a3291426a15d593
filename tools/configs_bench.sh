# The other BASELINE configs on one GPU (bench lines, one JSON per line):  bash tools/configs_bench.sh OUT
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${1:-$R/gpurun_out/configs.jsonl}
mkdir -p $R/gpurun_out && cd /tmp && export TMPDIR=/tmp
: > $OUT
for args in "--img 512 --backbone swin_t" "--img 1024 --backbone swin_s" "--img 1024 --backbone swin_s --grad-wire fp16" "--img 1024 --backbone swin_b"; do
  echo "== $args"
  timeout -k 10 300 python3 -u $R/bench.py --no-cpu-baseline --no-roofline --no-input-pipeline --steps 10 --warmup 6 $args >> $OUT 2> $R/gpurun_out/configs.err || { tail -20 $R/gpurun_out/configs.err; exit 1; }
  tail -1 $OUT | cut -c1-400
done

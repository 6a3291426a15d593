# kbench A/B over environment settings, interleaved:  bash tools/gpu_ab_env.sh TAG MODE "A=1 B=2" "A=0" ...
# (each quoted argument is one arm's environment; the arms run in the given order)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
TAG=$1; MODE=$2; shift 2
for arm in "$@"; do
  echo "== $arm"
  env $arm timeout -k 10 150 python3 -u $R/tools/kbench.py $MODE 2>&1 | grep -v "Warn\|amdgpu.ids" || exit 1
done > $O/${TAG}_ab.log
cat $O/${TAG}_ab.log

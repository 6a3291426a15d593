# Time a kbench mode against the normal build and each ablation build: bash tools/exp_run.sh MODE SRC MASK...
R=${GRAFT_REPO_ROOT:-$(pwd)}
M=$1; SRC=$2; shift 2
cd /tmp && export TMPDIR=/tmp
echo "== base"; timeout -k 10 120 python3 -u $R/tools/kbench.py $M 2>&1 | grep -v "Warning\|amdgpu.ids" || exit 1
for X in "$@"; do
  echo "== exp $X"
  MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_${SRC}_$X.so timeout -k 10 120 python3 -u $R/tools/kbench.py $M 2>&1 | grep -v "Warning\|amdgpu.ids" || exit 1
done

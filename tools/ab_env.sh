# A/B a kbench mode with and without an env switch: bash tools/ab_env.sh MODE VAR=VAL
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
echo "== base"; timeout -k 10 200 python3 -u $R/tools/kbench.py $1 2>&1 | grep -v "Warning\|amdgpu.ids" || exit 1
echo "== $2"; env $2 timeout -k 10 200 python3 -u $R/tools/kbench.py $1 2>&1 | grep -v "Warning\|amdgpu.ids" || exit 1

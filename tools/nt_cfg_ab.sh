# NT GEMM ring configurations vs hipBLASLt at the stage 1-3 shapes: bash tools/nt_cfg_ab.sh CFG...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  echo "== MSU_NT_CFG=$c"
  MSU_NT_CFG=$c timeout -k 10 200 python3 -u $R/tools/kbench.py nt 2>&1 | grep -v "Warning\|amdgpu.ids" || exit 1
done

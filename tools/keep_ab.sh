# Attention with / without the stored dropout keep bits (kbench attn, stage 0): bash tools/keep_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for k in 1 0; do
  echo "== MSU_ATTN_KEEP=$k"
  MSU_ATTN_KEEP=$k timeout -k 10 200 python3 -u $R/tools/kbench.py attn 2>&1 | grep "stage0 res256 nh3 p=0.05" || exit 1
done; done

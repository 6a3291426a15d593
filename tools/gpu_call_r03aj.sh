# r03aj: one-pass Linear backward ring-depth / GELU'-load variants (tracked loads: correct by
# construction; timing only): a = 96x96 at D 4, b = GELU' at D 3, c = b + H loads on every wave,
# d = GELU' D 2 + H loads on every wave
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
L=$O/r03aj_linbwd_variants.log; : > $L
for rep in 1 2; do
  echo "== base" >> $L
  timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py 96 96 >> $L 2>&1 || exit 1
  timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py 384 96 1 >> $L 2>&1 || exit 1
  echo "== a" >> $L
  MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_linbwd_a.so timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py 96 96 >> $L 2>&1 || exit 1
  for v in b c d; do
    echo "== $v" >> $L
    MSU_LIB_OVERRIDE=$R/tools/exp/libmsunet_gemm_linbwd_$v.so timeout -k 10 120 python3 -u $R/tools/linbwd_bench.py 384 96 1 >> $L 2>&1 || exit 1
  done
done
grep "==\|linbwd" $L | sed 's/dgrad.*//'

# NT GEMM per-shape timing, this build vs an override library (NT_B)
R=${GRAFT_REPO_ROOT:-$PWD}
for L in "" "$NT_B"; do
  echo "== lib ${L:-this build}"
  for shp in "32768 1152 384" "32768 384 1536" "32768 384 384" "131072 576 192" "131072 192 768" "8192 2304 768" "8192 768 3072" "32768 1536 384"; do
    MSU_LIB_OVERRIDE=$L timeout -k 10 60 python -u $R/tools/nt_one.py $shp 30 2>&1 | grep "nt M" || exit 3
  done
done

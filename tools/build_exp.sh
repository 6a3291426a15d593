# Ablation builds of one kernel source: bash tools/build_exp.sh SRC MASK... -> tools/exp/libmsunet_SRC_MASK.so
# (SRC compiled with -DMSU_EXP=MASK, linked with the other objects of the normal build).
# Load one with MSU_LIB_OVERRIDE=<path>; the results of such a build are WRONG by design.
set -e
R=$(cd $(dirname $0)/.. && pwd)
SRC=$1; shift
B=$R/semantic_segmentation_of_stylegan2_artifacts_amd/_build
mkdir -p $R/tools/exp
OTHERS=$(ls $B/*.o | grep -v "/$SRC.o$")
for M in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 -DMSU_EXP=$M $EXTRA \
     -c $R/semantic_segmentation_of_stylegan2_artifacts_amd/csrc/$SRC.hip -o /tmp/exp_${SRC}_$M.o &
done
wait
for M in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/exp/libmsunet_${SRC}_$M.so /tmp/exp_${SRC}_$M.o $OTHERS
  echo $R/tools/exp/libmsunet_${SRC}_$M.so
done

# Whole-library build with extra compiler flags, for same-box A/B runs (MSU_LIB_OVERRIDE=<path>):
#   bash tools/build_variant.sh NAME FLAG...   -> tools/exp/libmsunet_NAME.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
NAME=$1; shift
W=/tmp/msu_variant_$NAME
mkdir -p $W $R/tools/exp
for f in $R/semantic_segmentation_of_stylegan2_artifacts_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -munsafe-fp-atomics "$@" \
    -c $f -o $W/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/exp/libmsunet_$NAME.so $W/*.o
echo $R/tools/exp/libmsunet_$NAME.so

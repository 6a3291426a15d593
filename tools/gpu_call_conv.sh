# conv parity tests + kbench conv A/B over MSU_CONV_V values:  bash tools/gpu_call_conv.sh TAG "4 3 4 3"
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
TAG=$1
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ops.py -m gpu -q -k "conv" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/${TAG}_conv_tests.log 2>&1; rc=$?; echo "conv tests rc=$rc"; tail -2 $O/${TAG}_conv_tests.log; [ $rc -gt 1 ] && exit $rc
for v in $2; do echo "== v$v"; MSU_CONV_V=$v timeout -k 10 120 python3 -u $R/tools/kbench.py conv 2>&1 | grep -v "Warn\|amdgpu.ids" || exit 1; done > $O/${TAG}_conv_ab.log
cat $O/${TAG}_conv_ab.log

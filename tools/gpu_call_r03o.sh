# r03o: round evidence (tests, bench, step profile, conv / wgrad HBM counters, graph probe) +
# SQ counters of the v3 refine conv
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_round3.sh r03o || exit $?
MSU_CONV_V=3 CONV_V=3 bash $R/tools/pmc_conv3.sh r03o > $R/gpurun_out/r03o_pmc_conv3.log 2>&1; echo "pmc rc=$?"

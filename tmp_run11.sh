R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01j
mkdir -p $O
for dly in 20 5 60; do SRGNN_HUB_DISPATCH_DELAY_US=$dly timeout -k 10 300 python3 $R/tools/sweep.py --thresholds 32:-1,32:131072 --rounds 10 > $O/sweep_d$dly.json 2> $O/sweep_d$dly.err; done
echo "all rc=$?"

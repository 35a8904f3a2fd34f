R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01l
mkdir -p $O
timeout -k 10 400 python3 $R/tools/sweep.py --thresholds 32:131072:0,32:131072:16,32:131072:64,32:131072:256,32:131072:1024,32:131072:4096 --rounds 5 > $O/sweep_hot.json 2> $O/e3
echo "all rc=$?"

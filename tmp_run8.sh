R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01g
mkdir -p $O
timeout -k 10 900 python -m pytest $R/tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 300 python3 $R/tools/hub_latency.py > $O/hub_latency.json 2> $O/hub_latency.err
timeout -k 10 300 python3 $R/tools/sweep.py --thresholds 32:-1,32:65536,32:131072,32:16384 > $O/sweep.json 2> $O/sweep.err
echo "all rc=$?"

R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01h
mkdir -p $O
timeout -k 10 900 python -m pytest $R/tests/test_gpu_parity.py -m gpu -q -x > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
for A in 0 1 2; do SRGNN_HUB_ABLATION=$A timeout -k 10 300 python3 $R/tools/hub_latency.py > $O/hub_latency_abl$A.json 2> $O/hub_latency_abl$A.err; done
timeout -k 10 300 python3 $R/tools/sweep.py --thresholds 32:-1,32:131072,32:65536,32:16384 > $O/sweep.json 2> $O/sweep.err
echo "all rc=$?"

R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01i
mkdir -p $O
timeout -k 10 900 python -m pytest $R/tests -m gpu -q > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 600 python3 $R/bench.py --steps 5 --cpu-seconds 12 > $O/bench.json 2> $O/bench.err
echo "all rc=$?"

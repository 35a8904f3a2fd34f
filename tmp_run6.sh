R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01e
mkdir -p $O
timeout -k 10 900 python -m pytest $R/tests -m gpu -q > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log

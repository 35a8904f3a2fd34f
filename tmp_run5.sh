export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01d
mkdir -p $O
timeout -k 10 600 python -m pytest $R/tests/test_wavelet_gpu.py -m gpu -q > $O/pytest_wavelet.log 2>&1; echo "pytest rc=$?" >> $O/pytest_wavelet.log
timeout -k 10 600 python3 $R/tools/order_sweep.py --rcm > $O/order_sweep.json 2> $O/order_sweep.err
echo "all rc=$?"

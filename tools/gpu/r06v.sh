# round 6: one-launch fp64 steps with the fp64 hub rule -- wavelet parity
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06v
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py tests/test_shims_gpu.py > $O/pytest.log 2>&1

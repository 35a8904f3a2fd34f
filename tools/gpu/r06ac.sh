# round 6: the fp64 filter bank over the halo partition (virtual ranks) -- parity; the gloo GPU ranks
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ac
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py -k "halo" > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_dist_gpu_gloo.py > $O/pytest_gloo.log 2>&1

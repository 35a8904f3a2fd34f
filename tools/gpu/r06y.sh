# round 6: the full-size fp64 filter bank test (products, blocked plan, every row of two columns)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06y
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu tests/test_full_size_gpu.py -k "wavelet_f64 or arxiv" > $O/pytest.log 2>&1

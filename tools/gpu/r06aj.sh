# round 6: fp64 halo filter bank on ragged operators (empty rows, tiny ranks, odd panels)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06aj
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_wavelet_gpu.py -k "halo_wavelet_f64" > $O/tests.log 2>&1

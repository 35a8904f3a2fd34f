# round 6: fp64 steps over feature chunks -- parity, then the products sweep (chunk width x blocks)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/probes/cheby64_parts_probe.py products --plan --no-ref --configs 16::,8:::64,12:::64,16:::64,4:::32,6:::32,8:::32,12:::32 > $O/cw_sweep.json 2> $O/cw_sweep.err

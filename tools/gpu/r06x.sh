# round 6: the plain C host of the fp64 steps, and the C-API tests
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_capi.py > $O/pytest.log 2>&1

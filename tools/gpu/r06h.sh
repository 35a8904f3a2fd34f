# round 6: fp64 Chebyshev steps over column-blocked plans -- parity, then the products sweep
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06h
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py tests/test_capi.py tests/test_plan_gpu.py tests/test_plan_lifecycle_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/probes/cheby64_parts_probe.py products --plan > $O/cheby64_plan.json 2> $O/cheby64_plan.err

# round 6: planner whole-row limit option -- plan/wavelet parity, then the products fp64 sweep
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py tests/test_plan_gpu.py tests/test_plan_lifecycle_gpu.py tests/test_capi.py > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/probes/cheby64_parts_probe.py products --plan --no-ref --configs 16::,16::64,16::96,16::128,16::192,16::256,12::128,24::128 > $O/whole_sweep.json 2> $O/whole_sweep.err

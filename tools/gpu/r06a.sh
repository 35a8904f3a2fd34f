set -o pipefail
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_fake_rccl_gpu.py tests/test_plan_gpu.py tests/test_capi.py > $O/pytest_quick.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests/test_full_size_gpu.py -k "int64 or p8_partition" > $O/pytest_full.log 2>&1  &&
timeout -k 10 600 python -u bench.py --op wavelet --dtype f64 --steps 5 --warmup 1 > $O/wav64_products.json 2> $O/wav64_products.err

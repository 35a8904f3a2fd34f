# round 6: fused-step lean epilogue (fp64 and fp32 fused) -- parity, then the products fp64 bench
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06m
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py tests/test_capi.py tests/test_full_size_gpu.py -k "not papers100M and not rmat" > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench.py --op wavelet --dtype f64 --steps 5 --warmup 1 > $O/wav64_products.json 2> $O/wav64_products.err

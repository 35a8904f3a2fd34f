# round 6: the fp64 wavelet bench after the blocked steps (products; RMAT-26's widest block), its kernel trace
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06j
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_wavelet_gpu.py > $O/pytest_wavelet.log 2>&1 &&
timeout -k 10 600 python -u bench.py --op wavelet --dtype f64 --steps 5 --warmup 1 > $O/wav64_products.json 2> $O/wav64_products.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o wav64 --output-format csv -- python3 -u bench.py --op wavelet --dtype f64 --steps 3 --warmup 1 --pmc off --no-cpu-baseline > $O/wav64_prof.json 2> $O/wav64_prof.err

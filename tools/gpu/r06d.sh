# round 6: plan tests after the whole-hub-row launch, then the kernel-trace timelines and the default bench
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_plan_gpu.py tests/test_plan_lifecycle_gpu.py tests/test_aggregate_gpu.py tests/test_capi.py tests/test_fast_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_products.json 2> $O/bench_products.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tp -o tp --output-format csv -- python3 $R/bench.py --config products --steps 3 --warmup 2 --no-cpu-baseline --pmc off > $O/trace_products.json 2> $O/trace_products.err &&
python3 $R/tools/trace_timeline.py $O/tp --last 60 > $O/products_timeline.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ta -o ta --output-format csv -- python3 $R/bench.py --config arxiv --steps 10 --warmup 3 --no-cpu-baseline --pmc off > $O/trace_arxiv.json 2> $O/trace_arxiv.err &&
python3 $R/tools/trace_timeline.py $O/ta --last 40 > $O/arxiv_timeline.txt

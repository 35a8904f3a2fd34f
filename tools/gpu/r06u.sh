# round 6: the whole GPU suite after the planner sort moved off hipcub, smoke, the default bench
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06u
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu tests > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_products.json 2> $O/bench_products.err

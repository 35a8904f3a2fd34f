#!/bin/bash
# GPU-box script (round 5): the native planner -- its GPU tests, the plain-C example on products (and a
# kernel trace of it: the build's kernels), and the products bench.  Usage: r05_plan.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash "$R/tools/gpu/run_tests.sh" "$T" "$R/tests/test_plan_gpu.py" "$R/tests/test_gpu_parity.py" &&
timeout -k 10 200 python -u "$R/tools/dump_graph.py" --config products --out /tmp/products.csr > "$O/dump.txt" 2>&1 &&
timeout -k 10 200 "$R/examples/plan_propagate" /tmp/products.csr 128 10 10 > "$O/plan_example.json" 2> "$O/plan_example.err" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/extrace" -o ex --output-format csv -- "$R/examples/plan_propagate" /tmp/products.csr 128 10 10 > "$O/plan_example_traced.json" 2> "$O/plan_example_traced.err") &&
timeout -k 10 600 python -u "$R/bench.py" --steps 20 --warmup 5 > "$O/bench_products.json" 2> "$O/bench_products.err"

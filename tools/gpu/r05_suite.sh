#!/bin/bash
# GPU-box script (round 5): the whole GPU suite, the plain-C planner example on products and the
# products bench.  Usage: r05_suite.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash "$R/tools/gpu/run_tests.sh" "$T" &&
timeout -k 10 200 python -u "$R/tools/dump_graph.py" --config products --out /tmp/products.csr > "$O/dump.txt" 2>&1 &&
timeout -k 10 200 "$R/examples/plan_propagate" /tmp/products.csr 128 10 10 > "$O/plan_example.json" 2> "$O/plan_example.err" &&
timeout -k 10 600 python -u "$R/bench.py" --steps 20 --warmup 5 > "$O/bench_products.json" 2> "$O/bench_products.err"

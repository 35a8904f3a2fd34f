#!/bin/bash
# GPU-box script: the end-of-session evidence in one call, every step under its own time limit:
#   full pytest -m gpu, smoke(), rocprofv3 + PMC of the products hop (tools/gpu/profile.sh), and
#   bench.py on the products / arxiv configurations (JSON lines under gpurun_out/<tag>/); the
#   billion-edge ones go in a call of their own (bench_configs.sh TAG papers100M rmat26).
# Usage: final.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash "$R/tools/gpu/run_tests.sh" "$T" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 &&
bash "$R/tools/gpu/profile.sh" "$T" products > "$O/profile.txt" 2>&1 &&
bash "$R/tools/gpu/bench_configs.sh" "$T" "products:--steps 20 --warmup 5" "arxiv:--steps 20" \
    "products:--aggregate weighted --steps 10" "products:--op wavelet --steps 5"

#!/bin/bash
# GPU-box script: the medium-span halo mode's tests, then tools/halo_ranks.py at P = WORLDS with the
# mode on (default) and off, then the one-GPU products bench (regression check).
# Usage: medium_ab.sh TAG WORLDS [halo_ranks args...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; W=$2; shift 2
O=$R/gpurun_out/$T
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_parity.py -k "medium or rowacc or halo_virtual" $R/tests/test_halo_capi_gpu.py \
    -x -v --timeout 300 --timeout-method thread > $O/pytest_medium.log 2>&1 &&
timeout -k 10 600 python -u $R/tools/halo_ranks.py --worlds $W --chunks 6 "$@" > $O/halo_medium_on.json 2> $O/halo_medium_on.err &&
SRGNN_HALO_MEDIUM_SPANS=0 timeout -k 10 600 python -u $R/tools/halo_ranks.py --worlds $W --chunks 6 "$@" > $O/halo_medium_off.json 2> $O/halo_medium_off.err &&
timeout -k 10 600 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_products.json 2> $O/bench_products.err

#!/bin/bash
# GPU-box script (round 4): full GPU suite, products bench, one-shot layouts, RMAT-26 P = 8 per-rank hops.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash $R/tools/gpu/run_tests.sh $T &&
timeout -k 10 600 python $R/bench.py --steps 20 --warmup 5 > $O/bench_products.json 2> $O/bench_products.err &&
timeout -k 10 400 python $R/tools/one_shot_probe.py --config products --reps 3 > $O/one_shot_products.json 2> $O/one_shot_products.err &&
timeout -k 10 900 python -u $R/tools/halo_ranks.py --config rmat26 --worlds 8 --chunks 6 --quick --reps 3 > $O/halo_ranks_rmat26_p8.json 2> $O/halo_ranks_rmat26_p8.err

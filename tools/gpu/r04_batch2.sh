#!/bin/bash
# GPU-box script (round 4): full GPU suite, products bench A/B (staged packed-row entries vs not),
# one-shot layouts.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash $R/tools/gpu/run_tests.sh $T &&
bash $R/tools/gpu/lib_bench_ab.sh $T 2 scalable-roubust-gnn_amd/lib/libsrgnn_hip.so scalable-roubust-gnn_amd/lib/variants/libsrgnn_nostage.so &&
timeout -k 10 400 python $R/tools/one_shot_probe.py --config products --reps 3 > $O/one_shot_products.json 2> $O/one_shot_products.err

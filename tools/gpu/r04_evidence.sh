#!/bin/bash
# GPU-box script (round 4): the full GPU suite, smoke, the N = 2 bench over gloo on one GPU (device
# record + parity, whole-graph and sampled), and the end-to-end API timing on products.
# Usage: r04_evidence.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash $R/tools/gpu/run_tests.sh $T &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
SRGNN_DIST_BACKEND=gloo timeout -k 10 400 python $R/bench.py --gpus 2 --config arxiv --steps 3 --warmup 1 > $O/bench_arxiv_2ranks_gloo.json 2> $O/bench_arxiv_2ranks_gloo.err &&
SRGNN_DIST_BACKEND=gloo timeout -k 10 400 python $R/bench.py --gpus 2 --config arxiv --steps 3 --warmup 1 --dist-parity sampled > $O/bench_arxiv_2ranks_gloo_sampled.json 2> $O/bench_arxiv_2ranks_gloo_sampled.err &&
timeout -k 10 600 python $R/tools/e2e_api.py --config products --reps 3 > $O/e2e_api_products.json 2> $O/e2e_api_products.err

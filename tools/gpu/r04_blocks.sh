#!/bin/bash
# GPU-box script (round 4): products column blocks per hop beyond the automatic 8, two rounds.
# Usage: r04_blocks.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
for r in 1 2; do
  for B in 8 10 12; do
    bash $R/tools/gpu/ab_env_args.sh $T 1 "--steps 10 --warmup 2 --col-blocks $B" SRGNN_SPMM_WAVES=5 || exit 1
  done
done

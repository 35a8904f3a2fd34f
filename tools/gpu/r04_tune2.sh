#!/bin/bash
# GPU-box script (round 4): products whole-row length limit x column blocks, two rounds.
# Usage: r04_tune2.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
for r in 1 2; do
  for B in 6 7; do
    bash $R/tools/gpu/ab_env_args.sh $T 1 "--steps 10 --warmup 2 --col-blocks $B" SRGNN_BLOCK_WHOLE_MAX=32 SRGNN_BLOCK_WHOLE_MAX=48 SRGNN_BLOCK_WHOLE_MAX=64 SRGNN_BLOCK_WHOLE_MAX=96 || exit 1
  done
done

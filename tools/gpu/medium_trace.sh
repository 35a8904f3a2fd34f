#!/bin/bash
# GPU-box script: kernel trace + PMC of one P = 8 rank's hop compute (halo_trace.sh) with the
# medium-span mode, and halo_ranks at a few giant thresholds.  Usage: medium_trace.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1
O=$R/gpurun_out/$T
mkdir -p "$O"
bash $R/tools/gpu/halo_trace.sh $T 8 6 1 &&
for G in 4000 8000; do
  SRGNN_HALO_GIANT_THRESHOLD=$G timeout -k 10 600 python -u $R/tools/halo_ranks.py --worlds 8 --chunks 6 > $O/halo_giant$G.json 2> $O/halo_giant$G.err || exit 1
done

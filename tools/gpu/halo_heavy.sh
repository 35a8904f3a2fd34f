#!/bin/bash
# GPU-box script (round 4): the P = 8 halo chunks' slice-wave threshold (SRGNN_HEAVY_THRESHOLD) on products.
# Usage: halo_heavy.sh TAG THRESHOLD...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; shift; O=$R/gpurun_out/$T
mkdir -p "$O"
for H in "$@"; do
  SRGNN_HEAVY_THRESHOLD=$H timeout -k 10 200 python -u $R/tools/halo_ranks.py --config products --worlds 8 --chunks 6 --quick --reps 7 > $O/halo_h$H.json 2> $O/halo_h$H.err || exit 1
  grep "^P=8" $O/halo_h$H.err | sed "s/^/halo heavy $H: /" >> $O/ab.txt
done
cat $O/ab.txt

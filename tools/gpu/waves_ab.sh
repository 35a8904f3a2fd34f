#!/bin/bash
# GPU-box script (round 4): the row kernel's occupancy cap (SRGNN_SPMM_WAVES) on the products and arxiv
# benches (ab_env_args.sh) and on the products P = 8 per-rank hop (tools/halo_ranks.py --quick).
# Usage: waves_ab.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
bash $R/tools/gpu/ab_env_args.sh $1 1 "--steps 10 --warmup 2" SRGNN_SPMM_WAVES=5 SRGNN_SPMM_WAVES=0 SRGNN_SPMM_WAVES=6 SRGNN_SPMM_WAVES=4 &&
bash $R/tools/gpu/ab_env_args.sh $1 1 "--config arxiv --steps 50 --warmup 5" SRGNN_SPMM_WAVES=5 SRGNN_SPMM_WAVES=0 SRGNN_SPMM_WAVES=6 &&
for W in 5 0 6; do
  SRGNN_SPMM_WAVES=$W timeout -k 10 200 python -u $R/tools/halo_ranks.py --config products --worlds 8 --chunks 6 --quick --reps 7 > $O/halo_w$W.json 2> $O/halo_w$W.err || exit 1
  grep "^P=8" $O/halo_w$W.err | sed "s/^/waves $W: /" >> $O/ab.txt
done
cat $O/ab.txt

#!/bin/bash
# GPU-box script (round 4): products knob sweep after the slice-rule change -- column blocks per hop,
# whole-row length limit, occupancy cap -- and the P = 8 halo chunks' slice-wave threshold.
# Usage: r04_tune.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; O=$R/gpurun_out/$T
mkdir -p "$O"
for B in 6 5 7 8; do
  bash $R/tools/gpu/ab_env_args.sh $T 1 "--steps 10 --warmup 2 --col-blocks $B" SRGNN_SPMM_WAVES=5 || exit 1
done
bash $R/tools/gpu/ab_env_args.sh $T 1 "--steps 10 --warmup 2" SRGNN_BLOCK_WHOLE_MAX=16 SRGNN_BLOCK_WHOLE_MAX=48 SRGNN_SPMM_WAVES=6 SRGNN_SPMM_WAVES=0 || exit 1
for H in auto 300 1000; do
  SRGNN_HEAVY_THRESHOLD=$H timeout -k 10 200 python -u $R/tools/halo_ranks.py --config products --worlds 8 --chunks 6 --quick --reps 7 > $O/halo_h$H.json 2> $O/halo_h$H.err || exit 1
  grep "^P=8" $O/halo_h$H.err | sed "s/^/halo heavy $H: /" >> $O/ab.txt
done
cat $O/ab.txt

#!/bin/bash
# GPU-box script: P = 8 per-rank hop compute (tools/halo_ranks.py --quick) under a list of settings,
# each "NAME|ENV ASSIGNMENTS|halo_ranks args".  Usage: halo_knobs.sh TAG SETTING...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p "$O"
for S in "$@"; do
  N=$(echo "$S" | cut -d'|' -f1); E=$(echo "$S" | cut -d'|' -f2); A=$(echo "$S" | cut -d'|' -f3)
  env $E timeout -k 10 300 python -u $R/tools/halo_ranks.py --quick --reps 7 $A > $O/knob_$N.json 2> $O/knob_$N.err || exit 1
  echo "$N: $(grep 'P=' $O/knob_$N.err | grep -v rank | tail -1)" >> $O/knobs.txt
done

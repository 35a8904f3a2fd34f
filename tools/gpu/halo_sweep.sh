#!/bin/bash
# GPU-box script: tools/halo_ranks.py over chunk counts and hub thresholds (per-rank hop compute on
# one GPU).  Usage: halo_sweep.sh TAG WORLDS "ARGS1" "ARGS2" ...   (ARGS: extra halo_ranks.py flags)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; W=$2; shift 2; mkdir -p "$O"
i=0
for A in "$@"; do
  i=$((i + 1))
  timeout -k 10 400 python -u "$R/tools/halo_ranks.py" --worlds "$W" $A > "$O/halo_$i.json" 2> "$O/halo_$i.err" || exit 1
  python3 -c "
import json; d=json.load(open('$O/halo_$i.json'))
for P, w in d['worlds'].items():
    rs = w['ranks']
    print('$A', 'P', P, 'max compute', round(max(r['ms_compute'] for r in rs), 3), 'chunks', round(max(r['ms_chunks'] for r in rs), 3), 'hub', round(max(r['ms_hub'] for r in rs), 3), 'hub rows', max(r['hub_rows'] for r in rs))
" | tee -a "$O/summary.txt"
done

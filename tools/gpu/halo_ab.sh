#!/bin/bash
# GPU-box script: tools/halo_ranks.py (per-rank hop compute on one GPU) for library builds given as
# paths relative to the repo root.  Usage: halo_ab.sh TAG WORLDS LIB...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; W=$2; shift 2; mkdir -p "$O"
for L in "$@"; do
  v=$(basename "$L" .so)
  SRGNN_HIP_LIB=$R/$L timeout -k 10 400 python -u "$R/tools/halo_ranks.py" --worlds "$W" --chunks 6 > "$O/halo_$v.json" 2> "$O/halo_$v.err" || exit 1
done

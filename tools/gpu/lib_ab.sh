#!/bin/bash
# GPU-box script: bitwise check (hop_breakdown sha) and bench.py A/B of two builds of the library.
# Usage: lib_ab.sh TAG ROUNDS LIB_A LIB_B CONFIG...   (LIB_*: paths relative to the repo root)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=$1; ROUNDS=$2; A=$R/$3; B=$R/$4; shift 4
O=$R/gpurun_out/$TAG; mkdir -p "$O"
for C in "$@"; do
  for L in "$A" "$B"; do
    SRGNN_HIP_LIB=$L timeout -k 10 300 python "$R/tools/hop_breakdown.py" --config "$C" --reps 20 > "$O/hb_${C}_$(basename $L .so).json" 2> "$O/hb.err" || { cat "$O/hb.err"; exit 1; }
  done
  bash "$R/tools/gpu/ab_env.sh" "$TAG" "$ROUNDS" "$C" "SRGNN_HIP_LIB=$A" "SRGNN_HIP_LIB=$B" || exit 1
done

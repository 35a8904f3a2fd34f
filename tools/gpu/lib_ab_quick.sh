#!/bin/bash
# GPU-box script: the default bench without counter passes (--pmc off) for library builds given as paths
# relative to the repo root, alternated ROUNDS times.  Usage: lib_ab_quick.sh TAG ROUNDS "BENCH ARGS" LIB...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; N=$2; ARGS=$3; shift 3; mkdir -p "$O"
for r in $(seq 1 "$N"); do
  for L in "$@"; do
    v=$(basename "$L" .so)
    SRGNN_HIP_LIB=$R/$L timeout -k 10 300 python "$R/bench.py" $ARGS --no-cpu-baseline --pmc off > "$O/$v.json" 2> "$O/$v.err" || { tail -5 "$O/$v.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$v.json')); r=d['roofline']
print('$v', round(d['ms_per_step'],3), round(r['kernel_ms'],4), round(d['value']/1e9,3), 'exact', d['parity_vs_oracle']['bit_exact'])" | tee -a "$O/ab.txt"
  done
done

#!/bin/bash
# GPU-box script: bench.py A/B over environment settings, alternated ROUNDS times.
# Usage: ab_env.sh TAG ROUNDS CONFIG "ENV1" "ENV2" ...   (each ENV: space-free VAR=VALUE,VAR=VALUE list)
# BENCH_ARGS (environment): extra bench.py arguments, e.g. "--d 256"
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; ROUNDS=$2; C=$3; shift 3
mkdir -p "$O"
for r in $(seq 1 "$ROUNDS"); do
  for E in "$@"; do
    env $(echo "$E" | tr ',' ' ') timeout -k 10 300 python "$R/bench.py" --config "$C" --steps 5 --warmup 1 --no-cpu-baseline --pmc off $BENCH_ARGS > "$O/tmp.json" 2> "$O/tmp.err" || { cat "$O/tmp.err"; exit 1; }
    python3 -c "import json,sys; r=json.load(open('$O/tmp.json')); print('$C', '$BENCH_ARGS', '$E', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],4), round(r['value']/1e9,2))" | tee -a "$O/ab_$C.txt"
  done
done

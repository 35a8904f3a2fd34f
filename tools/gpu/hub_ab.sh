#!/bin/bash
# GPU-box script: hub-row latency (tools/hub_latency.py, bitwise against the slice path) for library
# builds given as paths relative to the repo root, then the hub / bit-exact GPU tests on the default build.
# Usage: hub_ab.sh TAG LIB...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; shift; mkdir -p "$O"
for L in "$@"; do
  v=$(basename "$L" .so)
  SRGNN_HIP_LIB=$R/$L timeout -k 10 240 python -u "$R/tools/hub_latency.py" > "$O/hub_$v.json" 2> "$O/hub_$v.err" || exit 1
done
timeout -k 10 400 python -u -m pytest "$R/tests" -m gpu -q -x -k "hub or products_timed or golden or bit_exact" \
    -p no:cacheprovider > "$O/pytest_hub.txt" 2>&1

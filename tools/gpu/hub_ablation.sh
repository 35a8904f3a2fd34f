#!/bin/bash
# GPU-box script: tools/hub_latency.py under each SRGNN_HUB_ABLATION mode -> gpurun_out/<tag>/
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
for A in ${ABLS:-0 1 2 3 4 5 6}; do
    SRGNN_HUB_ABLATION=$A timeout -k 10 300 python "$R/tools/hub_latency.py" > "$O/hub_latency_abl$A.json" 2> "$O/hub_latency_abl$A.err" || exit 1
done

#!/bin/bash
# GPU-box script: hop breakdown (tools/hop_breakdown.py) per light-row packing setting and heavy threshold.
# Usage: packed_sweep.sh TAG "LR:U:HEAVY ..." config...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; shift
SETS=$1; shift
mkdir -p "$O"
for C in "$@"; do
  for S in $SETS; do
    IFS=: read LR U H <<< "$S"
    SRGNN_PACKED_ROWS=$LR SRGNN_PACKED_U=$U SRGNN_HEAVY_THRESHOLD=$H timeout -k 10 200 python "$R/tools/hop_breakdown.py" --config "$C" --reps 20 >> "$O/sweep_$C.jsonl" || exit 1
  done
done
python3 - "$O" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/sweep_*.jsonl")):
    for line in open(f):
        r = json.loads(line)
        e = r["env"]
        print(r["config"], e.get("SRGNN_PACKED_ROWS"), e.get("SRGNN_PACKED_U"), e.get("SRGNN_HEAVY_THRESHOLD"),
              "full %.4f slice %.4f row %.4f" % (r["full_ms"], r.get("slice_ms", 0), r.get("row_ms", 0)), r["full_sha256"])
PY

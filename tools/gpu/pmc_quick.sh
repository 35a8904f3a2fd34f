#!/bin/bash
# GPU-box script: FETCH_SIZE and TCC hit/miss of tools/spmm_probe.py under an environment setting.
# Usage: pmc_quick.sh TAG CONFIG [VAR=VALUE ...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; C=$2; shift 2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o f --output-format csv -- python3 $R/tools/spmm_probe.py --config $C > $O/probe.json 2> $O/pf.err &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/ph -o h --output-format csv -- python3 $R/tools/spmm_probe.py --config $C > /dev/null 2> $O/ph.err &&
python3 - "$O" <<'PY'
import csv, glob, sys
o = sys.argv[1]
def rows(pat):
    f = glob.glob(o + pat, recursive=True)[0]
    return [r for r in csv.DictReader(open(f)) if "k_spmm<" in r.get("Kernel_Name", "") and "hub" not in r.get("Kernel_Name", "")]
f = rows("/pf/**/*counter_collection.csv")
h = rows("/ph/**/*counter_collection.csv")
fetch = [float(r["Counter_Value"]) for r in f if r["Counter_Name"] == "FETCH_SIZE"]
hit = [float(r["Counter_Value"]) for r in h if r["Counter_Name"] == "TCC_HIT_sum"]
miss = [float(r["Counter_Value"]) for r in h if r["Counter_Name"] == "TCC_MISS_sum"]
print("launches", len(fetch), "fetch_GB_per_launch(x2 gfx950)", round(2 * sum(fetch) / len(fetch) * 1024 / 1e9, 2),
      "l2_hit", round(sum(hit) / (sum(hit) + sum(miss)), 3), "miss_GB", round(sum(miss) * 128 / len(miss) / 1e9, 2))
PY

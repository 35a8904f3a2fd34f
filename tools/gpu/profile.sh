#!/bin/bash
# GPU-box script: the profiles committed under profiles/ for one bench configuration.
#   1. rocprofv3 --kernel-trace --stats of bench.py (per-kernel average durations)
#   2. separate --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_HIT/MISS) of tools/spmm_probe.py, folded into
#      HBM bytes per launch by tools/pmc_traffic.py (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction)
# Usage: profile.sh TAG [config]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1
C=${2:-products}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 $R/bench.py --config $C --steps 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o f --output-format csv -- python3 $R/tools/spmm_probe.py --config $C > $O/probe.json 2> $O/pf.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o w --output-format csv -- python3 $R/tools/spmm_probe.py --config $C > /dev/null 2> $O/pw.err &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/ph -o h --output-format csv -- python3 $R/tools/spmm_probe.py --config $C > /dev/null 2> $O/ph.err &&
python3 $R/tools/pmc_traffic.py --fetch $O/pf --write $O/pw --hits $O/ph --probe $O/probe.json --out $O/pmc_$C.json > /dev/null &&
python3 - "$O" <<'PY'
import csv, glob, sys
o = sys.argv[1]
f = glob.glob(o + "/trace/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in rows[:8]:
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY

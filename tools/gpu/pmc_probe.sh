#!/bin/bash
# GPU-box script: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_HIT/MISS) of
# tools/spmm_probe.py with the given probe arguments, folded by tools/pmc_traffic.py into HBM bytes
# per hop (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) -> gpurun_out/<tag>/pmc_<name>.json
# Usage: pmc_probe.sh TAG NAME [spmm_probe.py args...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1/$2; N=$2; shift 2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o f --output-format csv -- python3 $R/tools/spmm_probe.py "$@" > $O/probe.json 2> $O/pf.err &&
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o w --output-format csv -- python3 $R/tools/spmm_probe.py "$@" > /dev/null 2> $O/pw.err &&
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/ph -o h --output-format csv -- python3 $R/tools/spmm_probe.py "$@" > /dev/null 2> $O/ph.err &&
python3 $R/tools/pmc_traffic.py --fetch $O/pf --write $O/pw --hits $O/ph --probe $O/probe.json --out $R/gpurun_out/$(basename $(dirname $O))/pmc_$N.json

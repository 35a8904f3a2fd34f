#!/bin/bash
# GPU-box script: per-launch HBM traffic and duration of the products hop (its 9 launches: block 0's
# cut spans, the whole rows, blocks 1..7) -- rocprofv3 FETCH_SIZE / WRITE_SIZE passes and a kernel
# trace of tools/spmm_probe.py, summed by position in the hop.  Usage: hop_launch_pmc.sh TAG [probe args]
# (CYCLE, environment: launches per hop, default 9)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $O/hl_$C -o p --output-format csv -- python3 $R/tools/spmm_probe.py --reps 5 "$@" > $O/hl_probe.json 2> $O/hl_$C.err || exit 1
  python3 $R/tools/pmc_sum.py $O/hl_$C $C --per delay --cycle ${CYCLE:-9} >> $O/hop_launch_pmc.jsonl || exit 1
  rm -rf $O/hl_$C
done
timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/hl_tr -o t --output-format csv -- python3 $R/tools/spmm_probe.py --reps 5 "$@" > /dev/null 2> $O/hl_tr.err || exit 1
python3 $R/tools/trace_timeline.py $O/hl_tr --last 40 --only spmm,hub,delay > $O/hop_launch_trace.txt && rm -rf $O/hl_tr

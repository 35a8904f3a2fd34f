#!/bin/bash
# GPU-box script: where one P-rank halo hop's compute goes, on one GPU (virtual rank): a
# rocprofv3 kernel trace of op.compute (tools/halo_trace_probe.py) for the given ranks, the PMC
# traffic of that compute per hop (FETCH_SIZE, WRITE_SIZE, TCC hit/miss passes), and
# tools/halo_ranks.py for every rank.  Usage: halo_trace.sh TAG WORLD CHUNKS RANK... (env passes through)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=$1; W=$2; C=$3; shift 3
O=$R/gpurun_out/$T
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for RK in "$@"; do
  timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/tr$RK -o t --output-format csv -- python3 $R/tools/halo_trace_probe.py --world $W --rank $RK --chunks $C --reps 10 > $O/trace_r$RK.txt 2>&1 || exit 1
  python3 $R/tools/trace_timeline.py $O/tr$RK --last 60 >> $O/trace_r$RK.txt || exit 1
  rm -rf $O/tr$RK
  for CT in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $CT | cut -d' ' -f1)
    timeout -s KILL 300 rocprofv3 --pmc $CT -d $O/pmc$RK$tag -o p --output-format csv -- python3 $R/tools/halo_trace_probe.py --world $W --rank $RK --chunks $C --reps 10 > /dev/null 2> $O/pmc$RK$tag.err || exit 1
    for c in $CT; do python3 $R/tools/pmc_sum.py $O/pmc$RK$tag $c >> $O/pmc_r$RK.jsonl || exit 1; done
    rm -rf $O/pmc$RK$tag
  done
done
timeout -k 10 600 python -u $R/tools/halo_ranks.py --worlds $W --chunks $C > $O/halo_ranks_p$W.json 2> $O/halo_ranks_p$W.err

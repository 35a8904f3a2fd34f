#!/bin/bash
# GPU-box script: bench.py on the given configs, one JSON line each under gpurun_out/<tag>/.
# Usage: bench_configs.sh TAG "config[:extra args]" ...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p "$O"
for spec in "$@"; do
    cfg=${spec%%:*}; extra=""
    [ "$spec" != "$cfg" ] && extra=${spec#*:}
    echo "== $cfg $extra" >&2
    timeout -k 10 900 python "$R/bench.py" --config "$cfg" $extra > "$O/bench_$cfg.json" 2> "$O/bench_$cfg.err" || { echo "bench $cfg rc=$?" >&2; exit 1; }
    cat "$O/bench_$cfg.json"
done

#!/bin/bash
# GPU-box script: bench.py on the given configs, one JSON line each under gpurun_out/<tag>/.
# Usage: bench_configs.sh TAG "config[:extra args]" ...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p "$O"
i=0
for spec in "$@"; do
    cfg=${spec%%:*}; extra=""
    [ "$spec" != "$cfg" ] && extra=${spec#*:}
    tag=$(echo "$cfg $extra" | tr -c 'A-Za-z0-9\n' '_' | sed 's/__*/_/g; s/_$//')
    i=$((i + 1))
    echo "== $cfg $extra" >&2
    timeout -k 10 900 python "$R/bench.py" --config "$cfg" $extra > "$O/bench_${i}_$tag.json" 2> "$O/bench_${i}_$tag.err" || { echo "bench $cfg rc=$?" >&2; exit 1; }
    cat "$O/bench_${i}_$tag.json"
done

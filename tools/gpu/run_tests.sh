#!/bin/bash
# GPU-box script: pytest -m gpu (whole suite, or the given test paths), log under gpurun_out/<tag>/.
# Usage: run_tests.sh TAG [test paths / pytest args]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p "$O"
[ $# -eq 0 ] && set -- "$R/tests"
timeout -k 10 1000 python -m pytest "$@" -m gpu -q -x -p no:cacheprovider -rA > "$O/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$O/pytest_gpu.log"
exit $rc

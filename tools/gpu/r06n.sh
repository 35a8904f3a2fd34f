# round 6: RMAT-26 fp64 blocked steps -- column blocks / whole-hub sweep on a 64-column block
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06n
mkdir -p $O
cd $R
timeout -k 10 900 python -u tools/probes/cheby64_parts_probe.py rmat26 --d 64 --plan --no-ref --configs 4:,8:,12:,16:,24:,8:131072 > $O/rmat26_plan.json 2> $O/rmat26_plan.err

# round 6: RMAT-26 fp64 halo ranks over the planner-blocked per-rank plans (against r06ae's one launch)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ah
mkdir -p $O
cd $R
timeout -k 10 900 python -u tools/probes/halo_cheby64_ranks.py --config rmat26 --world 8 --d 64 --reps 2 --blocks 0 > $O/rmat26_p8_auto.json 2> $O/rmat26_p8_auto.err

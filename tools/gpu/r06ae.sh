# round 6: per-rank compute of the fp64 filter bank over the halo partition (every rank's share on one GPU)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ae
mkdir -p $O
cd $R
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 > $O/products_p8.json 2> $O/products_p8.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 4 > $O/products_p4.json 2> $O/products_p4.err &&
timeout -k 10 900 python -u tools/probes/halo_cheby64_ranks.py --config rmat26 --world 8 --d 64 --reps 2 > $O/rmat26_p8.json 2> $O/rmat26_p8.err

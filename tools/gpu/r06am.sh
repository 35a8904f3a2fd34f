# round 6: where the chunked fp64 order's time goes (per chunk, and the halo plan's groups as launches)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06am
mkdir -p $O
cd $R
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 --chunks 6 > $O/products_p8_c6.json 2> $O/products_p8_c6.err

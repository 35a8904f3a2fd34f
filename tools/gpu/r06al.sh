# round 6: per-rank compute of the GPU ranks' overlapped fp64 order (one launch per row chunk) vs one launch
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06al
mkdir -p $O
cd $R
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 --chunks 6 > $O/products_p8_c6.json 2> $O/products_p8_c6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 4 --chunks 6 > $O/products_p4_c6.json 2> $O/products_p4_c6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 2 --chunks 4 > $O/products_p2_c4.json 2> $O/products_p2_c4.err

# round 6: the fp64 halo wavelet's per-rank one-launch order at P=2 (against r06af's blocked plans)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ag
mkdir -p $O
cd $R
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 2 --blocks 1 > $O/products_p2_b1.json 2> $O/products_p2_b1.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 --blocks 4 > $O/products_p8_b4.json 2> $O/products_p8_b4.err

# round 6: fp64 halo overlapped orders with the hub group rows above 2048 entries as hub workgroups -- tests, per-rank timing
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ar
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_dist_gpu_gloo.py tests/test_wavelet_gpu.py -k "wavelet or nojoin" > $O/tests.log 2>&1 &&
timeout -k 10 900 python -u tools/probes/halo_cheby64_ranks.py --config rmat26 --world 8 --d 64 --reps 2 --chunks 6 > $O/rmat26_p8_g6.json 2> $O/rmat26_p8_g6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 --chunks 6 > $O/products_p8_g6.json 2> $O/products_p8_g6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 4 --chunks 6 > $O/products_p4_g6.json 2> $O/products_p4_g6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 2 --chunks 4 > $O/products_p2_g4.json 2> $O/products_p2_g4.err

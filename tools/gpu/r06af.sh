# round 6: the fp64 halo wavelet over per-rank column-blocked plans -- parity, then per-rank timing (auto and forced)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06af
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_wavelet_gpu.py -k "halo_wavelet_f64" > $O/tests.log 2>&1 &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 4 > $O/products_p4_auto.json 2> $O/products_p4_auto.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 4 --blocks 8 > $O/products_p4_b8.json 2> $O/products_p4_b8.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 > $O/products_p8_auto.json 2> $O/products_p8_auto.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 2 > $O/products_p2_auto.json 2> $O/products_p2_auto.err

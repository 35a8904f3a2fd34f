# round 6: fp64 halo orders overlapped per exchange group (hub group first) -- GPU-rank tests, per-rank timing,
# the N=2 fp64 wavelet bench path (two ranks on one GPU over gloo)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06an
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_dist_gpu_gloo.py tests/test_wavelet_gpu.py -k "wavelet" > $O/tests.log 2>&1 &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 8 --chunks 6 > $O/products_p8_g6.json 2> $O/products_p8_g6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 4 --chunks 6 > $O/products_p4_g6.json 2> $O/products_p4_g6.err &&
timeout -k 10 500 python -u tools/probes/halo_cheby64_ranks.py --config products --world 2 --chunks 4 > $O/products_p2_g4.json 2> $O/products_p2_g4.err &&
SRGNN_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --op wavelet --dtype f64 --steps 2 --warmup 1 > $O/wav64_n2_gloo.json 2> $O/wav64_n2_gloo.err

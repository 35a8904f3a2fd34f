# round 6: the N = 2 wavelet bench path (fp32 and fp64) under torch.distributed.run, two ranks on one GPU (gloo)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ad
mkdir -p $O
cd $R
SRGNN_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --op wavelet --dtype f64 --steps 2 --warmup 1 > $O/wav64_n2_gloo.json 2> $O/wav64_n2_gloo.err &&
SRGNN_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --op wavelet --steps 2 --warmup 1 > $O/wav32_n2_gloo.json 2> $O/wav32_n2_gloo.err

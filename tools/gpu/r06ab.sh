# round 6: the N > 1 bench path as the driver launches it (torch.distributed.run), two ranks sharing one
# GPU over gloo (the dry run of the halo-exchange path; RCCL needs one GPU per rank)
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ab
mkdir -p $O
cd $R
SRGNN_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err

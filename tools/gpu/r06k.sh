# round 6: the fp64 filter bank on RMAT-26's widest column block (blocked fp64 steps), PMC roofline
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06k
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1120 python -u bench.py --op wavelet --dtype f64 --config rmat26 --steps 2 --warmup 1 > $O/wav64_rmat26.json 2> $O/wav64_rmat26.err

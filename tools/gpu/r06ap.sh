# round 6: the final tree after SRG_CHEBY_HUB_NOJOIN -- full GPU suite, smoke(), the default bench line,
# then RMAT-26 P=8 fp64 halo ranks per exchange group
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/r06ap
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 900 python -u tools/probes/halo_cheby64_ranks.py --config rmat26 --world 8 --d 64 --reps 2 --chunks 6 > $O/rmat26_p8_g6.json 2> $O/rmat26_p8_g6.err
